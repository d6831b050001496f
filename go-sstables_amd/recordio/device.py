"""Device-resident decode (torch tensors as HBM buffers) over rio_device_decode.

torch is plumbing here (allocation, streams, events); every byte of decode work is done by the
HIP kernels of librio.so.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import torch

from . import _lib as L


@dataclass
class DecodeBuffers:
    out: torch.Tensor      # uint8 [>= total_out_bytes]
    out_off: torch.Tensor  # int64 [n + 1]
    rec_off: torch.Tensor  # int64 [n]
    flags: torch.Tensor    # uint8 [n]
    info: torch.Tensor     # uint8 [sizeof(rio_file_info)]


INFO_BYTES = ctypes.sizeof(L.FileInfo)


def to_device_file(image, device: int = 0) -> tuple[torch.Tensor, int]:
    """Copy a file image (bytes / numpy uint8) into HBM with RIO_DEVICE_PAD readable pad bytes."""
    import numpy as np

    n = len(image)
    t = torch.zeros(n + L.RIO_DEVICE_PAD, dtype=torch.uint8, device=f"cuda:{device}")
    if n:
        import warnings

        arr = np.frombuffer(image, dtype=np.uint8) if isinstance(image, (bytes, bytearray)) else image
        with warnings.catch_warnings():  # a read-only source (bytes) is only read by the H2D copy
            warnings.simplefilter("ignore", UserWarning)
            src = torch.from_numpy(np.ascontiguousarray(arr))
        t[:n].copy_(src)
    return t, n


def header_codec(img) -> int | None:
    """The compression type in a file image's 8-byte header (readFileHeaderFromBuffer,
    common_reader.go:22-44: version, then the compression type from version 2 on), as the decode's
    codec hint; None when the header is short, older or names no codec the device decodes."""
    if len(img) < 8:
        return None
    version = int.from_bytes(bytes(img[0:4]), "little")
    comp = int.from_bytes(bytes(img[4:8]), "little")
    return comp if version >= 2 and comp <= 3 else None


class DeviceDecoder:
    def __init__(self, device: int = 0, own_ctx: bool = False):
        """own_ctx: a context of its own (rio_ctx_create) instead of the device's shared default one, so
        several decoders on one device can be driven from different host threads."""
        self.device = device
        if own_ctx:
            h = ctypes.c_void_p()
            rc = L.lib().rio_ctx_create(device, ctypes.byref(h))
            if rc != L.RIO_OK:
                raise RuntimeError(f"rio_ctx_create(device={device}): {L.strerror(rc)}")
            self.ctx, self._own = h.value, True
        else:
            self.ctx, self._own = L.default_ctx(device), False

    def __del__(self):
        if getattr(self, "_own", False) and self.ctx:
            L.lib().rio_ctx_destroy(self.ctx)
            self.ctx = None

    def alloc(self, n_records: int, total_bytes: int) -> DecodeBuffers:
        dev = f"cuda:{self.device}"
        return DecodeBuffers(
            out=torch.empty(max(total_bytes, 1) + 16, dtype=torch.uint8, device=dev),
            out_off=torch.empty(n_records + 1, dtype=torch.int64, device=dev),
            rec_off=torch.empty(max(n_records, 1), dtype=torch.int64, device=dev),
            flags=torch.empty(max(n_records, 1), dtype=torch.uint8, device=dev),
            info=torch.zeros(INFO_BYTES, dtype=torch.uint8, device=dev),
        )

    def launch(self, d_file: torch.Tensor, length: int, b: DecodeBuffers, stream=None, comp=None) -> None:
        """Enqueue the whole decode on `stream` (default: torch's current stream); no host sync.
        `comp`: the file header's compression type when the caller knows it (only that codec's
        kernels are launched: rio_device_decode_ex)."""
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        rc = L.lib().rio_device_decode_ex(
            self.ctx, d_file.data_ptr(), length, L.RIO_COMP_UNKNOWN if comp is None else comp, b.out.data_ptr(),
            b.out.numel(), b.out_off.data_ptr(), b.rec_off.data_ptr(), b.flags.data_ptr(), b.out_off.numel() - 1,
            b.info.data_ptr(), ctypes.c_void_p(s.cuda_stream))
        if rc != L.RIO_OK:
            raise RuntimeError(f"rio_device_decode: {L.strerror(rc)}")

    @staticmethod
    def info(b: DecodeBuffers) -> dict:
        raw = bytes(b.info.cpu().numpy().tobytes())
        return L.FileInfo.from_buffer_copy(raw).as_dict()

    def launch_batch(self, files: list, bufs: list, stream=None) -> None:
        """Enqueue rio_device_decode_batch for [(d_file, length)] into the matching DecodeBuffers."""
        import numpy as np

        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        n = len(files)
        p = lambda xs: np.array(xs, dtype=np.uint64)  # noqa: E731
        arrs = [p([f.data_ptr() for f, _ in files]), p([ln for _, ln in files]), p([b.out.data_ptr() for b in bufs]),
                p([b.out.numel() for b in bufs]), p([b.out_off.data_ptr() for b in bufs]),
                p([b.rec_off.data_ptr() for b in bufs]), p([b.flags.data_ptr() for b in bufs]),
                p([b.out_off.numel() - 1 for b in bufs]), p([b.info.data_ptr() for b in bufs])]
        rc = L.lib().rio_device_decode_batch(self.ctx, n, *[a.ctypes.data for a in arrs], ctypes.c_void_p(s.cuda_stream))
        if rc != L.RIO_OK:
            raise RuntimeError(f"rio_device_decode_batch: {L.strerror(rc)}")

    def decode_batch(self, files: list, stream=None):
        """Size every file's outputs with capacity-0 probes (one batch call), then decode the batch.
        Returns [(buffers, info)] in file order."""
        bufs = [self.alloc(0, 0) for _ in files]
        # a gzip record of several members is larger than the framing's size: its decode asks again
        for _ in range(3):
            self.launch_batch(files, bufs, stream)
            torch.cuda.synchronize(self.device)
            infos = [self.info(b) for b in bufs]
            if all(i["status"] != L.RIO_ERR_CAPACITY for i in infos):
                break
            bufs = [self.alloc(i["n_records"], i["total_out_bytes"]) if i["status"] == L.RIO_ERR_CAPACITY else b
                    for b, i in zip(bufs, infos)]
        return [(b, self.info(b)) for b in bufs]

    def decode(self, d_file: torch.Tensor, length: int, stream=None, comp=None):
        """Size the outputs with a capacity-0 probe, then decode. Returns (buffers, info)."""
        b = self.alloc(0, 0)
        # (a gzip record of several members is larger than the framing's size: the decode asks again)
        for _ in range(3):
            self.launch(d_file, length, b, stream, comp)
            torch.cuda.synchronize(self.device)
            info = self.info(b)
            if info["status"] != L.RIO_ERR_CAPACITY:
                break
            b = self.alloc(info["n_records"], info["total_out_bytes"])
        return b, info

    def stage_ms(self):
        """Mean walk / scan / placement / decode milliseconds of the calls recorded since rio_ctx_set_timing
        (empty while timing is off, the context's default)."""
        ms = (ctypes.c_float * 4)()
        n = L.lib().rio_ctx_last_stage_ms(self.ctx, ms, 4)
        return list(ms)[:n]
