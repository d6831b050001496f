"""MI355X-native recordio decode — Python mirror of github.com/thomasjungblut/go-sstables/recordio.

Reader API (ReaderI / ReadAtI) and constants follow recordio/recordio.go; all decoding runs in the
HIP kernels of librio.so (go-sstables_amd/csrc). See DESIGN.md and INTEGRATION.md.
"""
from .errors import (EOF, ErrCorrupt, ErrUnexpectedEOF, ErrVarintOverflow, GoError,  # noqa: F401
                     HeaderChecksumMismatchErr, MagicNumberMismatchErr, errors_is, errors_unwrap)
from .reader import (CompressionTypeGZIP, CompressionTypeLzw, CompressionTypeNone,  # noqa: F401
                     CompressionTypeSnappy, FileHeaderSizeBytes, FileReader, MMapReader, NewFileReader,
                     NewFileReaderWithPath, NewMemoryMappedReaderWithPath)
from .writer import FileWriter, NewFileWriter, encode_file, generate  # noqa: F401

MagicNumberSeparatorLong = 0x130691
MagicNumberSeparatorLongBytes = bytes([0x91, 0x8D, 0x4C])
Version1, Version2, Version3, Version4 = 1, 2, 3, 4
CurrentVersion = Version4
RecordHeaderV3MaxSizeBytes = 31
RecordHeaderV4MaxSizeBytes = 36
