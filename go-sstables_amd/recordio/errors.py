"""Go-style error values for the recordio mirror.

The reference returns `(value, error)` pairs and its tests use `errors.Is` / `errors.Unwrap` and
message substrings; this module gives the Python mirror the same shape so the parity tests read
like recordio/*_test.go. Sentinels follow common_reader.go:19-20 and the io package.
"""
from __future__ import annotations


class GoError(Exception):
    """An error value with an optional wrapped cause (fmt.Errorf("...: %w", err))."""

    def __init__(self, msg: str, wrapped: "GoError | None" = None):
        super().__init__(msg)
        self.msg = msg
        self.wrapped = wrapped

    def Error(self) -> str:  # noqa: N802 (Go naming)
        return self.msg

    def __str__(self) -> str:
        return self.msg

    def __repr__(self) -> str:
        return f"GoError({self.msg!r})"


def wrap(fmt_prefix: str, err: GoError) -> GoError:
    return GoError(f"{fmt_prefix}: {err.msg}", err)


def errors_is(err, target) -> bool:
    while err is not None:
        if err is target:
            return True
        err = getattr(err, "wrapped", None)
    return False


def errors_unwrap(err):
    return getattr(err, "wrapped", None)


EOF = GoError("EOF")
ErrUnexpectedEOF = GoError("unexpected EOF")
MagicNumberMismatchErr = GoError("magic number mismatch")
HeaderChecksumMismatchErr = GoError("header checksum mismatch")
ErrCorrupt = GoError("snappy: corrupt input")
ErrVarintOverflow = GoError("binary: varint overflows a 64-bit integer")
ErrUnsupported = GoError("not supported by the GPU decode path")
