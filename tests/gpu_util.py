"""Helpers for the GPU parity tests: run the device decode path and bring results to the host."""
import numpy as np
import torch

from recordio import _lib as L
from recordio.device import DeviceDecoder, to_device_file

_dec = None


def decoder():
    global _dec
    if _dec is None:
        _dec = DeviceDecoder(0)
    return _dec


def gpu_decode_arrays(image) -> dict:
    """Whole-file device decode (rio_device_decode) -> host numpy arrays + info."""
    d_file, n = to_device_file(image)
    b, info = decoder().decode(d_file, n)
    k, nb = info["n_records"], info["total_out_bytes"]
    res = dict(info)
    if info["status"] in (L.RIO_ERR_VERSION, L.RIO_ERR_COMPRESSION_TYPE, L.RIO_ERR_SHORT_FILE_HEADER) or (
            info["status"] == L.RIO_ERR_UNSUPPORTED and k == 0):
        return res
    res["out"] = b.out[:nb].cpu().numpy()
    res["out_off"] = b.out_off[:k + 1].cpu().numpy()
    res["rec_off"] = b.rec_off[:k].cpu().numpy()
    res["flags"] = b.flags[:k].cpu().numpy()
    return res


def assert_same_as_oracle(g: dict, o: dict, what=""):
    assert g["status"] == o["status"], (what, g["status"], o["status"])
    assert g["n_records"] == o["n_records"], (what, g["n_records"], o["n_records"])
    assert g["total_out_bytes"] == o["total_out_bytes"], what
    assert g["status_offset"] == o["status_offset"], (what, g["status_offset"], o["status_offset"])
    if o["status"] == L.RIO_ERR_HEADER_CRC:
        assert (g["detail0"], g["detail1"]) == (o["detail0"], o["detail1"]), what
    n = o["n_records"]
    np.testing.assert_array_equal(g["rec_off"][:n], o["rec_off"][:n], err_msg=what)
    np.testing.assert_array_equal(g["out_off"][:n + 1], o["out_off"][:n + 1], err_msg=what)
    np.testing.assert_array_equal(g["flags"][:n], o["flags"][:n], err_msg=what)
    if "first_bad" in g:
        assert (g["first_bad"], g["n_bad"]) == (o["first_bad"], o["n_bad"]), (what, g["first_bad"], o["first_bad"])
    if o["total_out_bytes"]:
        go, oo = g["out"], o["out"]
        bad = np.nonzero(o["flags"][:n] & (L.RIO_FLAG_CORRUPT | L.RIO_FLAG_EOF))[0]
        if bad.size:  # a record that does not decompress has unspecified bytes: compare the rest
            go, oo = go.copy(), oo.copy()
            for i in bad.tolist():
                lo, hi = int(o["out_off"][i]), int(o["out_off"][i + 1])
                go[lo:hi] = 0
                oo[lo:hi] = 0
        assert np.array_equal(go, oo), what


def gpu_available():
    try:
        return torch.cuda.is_available()
    except Exception:
        return False
