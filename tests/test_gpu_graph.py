"""rio_device_decode_ex captured into a HIP graph (include/rio.h: the device-resident call has no host
synchronisation and is graph-capturable): replaying the captured decode gives the oracle's records, and a
replay after new bytes of the same length were written into the captured file buffer decodes those bytes
(every launch reads the file, the sizes and the state from device memory, nothing is baked in at capture)."""
import numpy as np
import pytest

import oracle_py as orc
from gpu_util import assert_same_as_oracle

pytestmark = pytest.mark.gpu


def _arrays(b, info):
    k, nb = info["n_records"], info["total_out_bytes"]
    return dict(info, out=b.out[:nb].cpu().numpy(), out_off=b.out_off[: k + 1].cpu().numpy(),
                rec_off=b.rec_off[:k].cpu().numpy(), flags=b.flags[:k].cpu().numpy())


def _captured(dec, d_file, n, b, comp):
    import torch

    s = torch.cuda.Stream(device=0)
    # one launch on the capture stream first: the context then orders its calls on that stream alone
    dec.launch(d_file, n, b, s, comp)
    s.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        dec.launch(d_file, n, b, s, comp)
    return g, s


def _clear(b):
    b.out.zero_()
    b.out_off.zero_()
    b.rec_off.zero_()
    b.flags.fill_(0xFF)
    b.info.zero_()


@pytest.mark.parametrize("kind,comp", [(1, 2), (0, 2), (0, 0)], ids=["snappy-text", "snappy-literal", "none"])
def test_graph_replay_equals_the_oracle(kind, comp):
    import torch

    from recordio import generate
    from recordio.device import DeviceDecoder, to_device_file

    img = generate(20_000, 1024, comp, kind=kind, seed=11)
    dec = DeviceDecoder(0, own_ctx=True)
    d_file, n = to_device_file(img)
    b, info = dec.decode(d_file, n, comp=comp)
    g, s = _captured(dec, d_file, n, b, comp)
    _clear(b)
    torch.cuda.synchronize()
    with torch.cuda.stream(s):  # g.replay() launches on the current stream
        for _ in range(3):
            g.replay()
    torch.cuda.synchronize()
    got = _arrays(b, dec.info(b))
    assert_same_as_oracle(got, orc.file_reader_decode_arrays(np.asarray(img)), f"graph {kind}/{comp}")


def test_graph_replay_decodes_new_bytes_in_the_captured_buffer():
    import torch

    from recordio import generate
    from recordio.device import DeviceDecoder, to_device_file

    a = generate(5_000, 1024, 0, kind=0, seed=21)
    c = generate(5_000, 1024, 0, kind=0, seed=22)
    assert len(a) == len(c) and bytes(a) != bytes(c)
    dec = DeviceDecoder(0, own_ctx=True)
    d_file, n = to_device_file(a)
    b, _ = dec.decode(d_file, n, comp=0)
    g, s = _captured(dec, d_file, n, b, 0)
    for img in (c, a, c):
        d_file[:n].copy_(torch.from_numpy(np.asarray(img)))
        _clear(b)
        torch.cuda.synchronize()
        with torch.cuda.stream(s):
            g.replay()
        torch.cuda.synchronize()
        assert_same_as_oracle(_arrays(b, dec.info(b)), orc.file_reader_decode_arrays(np.asarray(img)), "graph new bytes")
