"""rio_device_decode_ex captured into a HIP graph (include/rio.h: the device-resident call has no host
synchronisation and is graph-capturable): replaying the captured decode gives the oracle's records, and a
replay after new bytes of the same length were written into the captured file buffer decodes those bytes
(every launch reads the file, the sizes and the state from device memory, nothing is baked in at capture). And the
per-stage timing events: off on a new context (rio_ctx_last_stage_ms gives nothing), recorded once rio_ctx_set_timing asks,
with the decode's results unchanged either way."""
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


def test_stage_timing_is_off_until_asked():
    import torch

    from recordio import _lib as L
    from recordio import generate
    from recordio.device import DeviceDecoder, to_device_file

    img = generate(20_000, 1024, 2, kind=1, seed=31)
    want = orc.file_reader_decode_arrays(np.asarray(img))
    dec = DeviceDecoder(0, own_ctx=True)
    d_file, n = to_device_file(img)
    b, info = dec.decode(d_file, n, comp=2)
    assert dec.stage_ms() == []
    assert L.lib().rio_ctx_set_timing(dec.ctx, 4) == L.RIO_OK
    s = torch.cuda.Stream(device=0)
    for _ in range(3):
        _clear(b)
        torch.cuda.synchronize()  # the clear runs on torch's stream, the decode on s
        dec.launch(d_file, n, b, s, 2)
    torch.cuda.synchronize()
    ms = dec.stage_ms()
    assert len(ms) == 4 and all(x > 0 for x in ms), ms
    assert_same_as_oracle(_arrays(b, dec.info(b)), want, "timed")
    assert L.lib().rio_ctx_set_timing(dec.ctx, 0) == L.RIO_OK
    _clear(b)
    torch.cuda.synchronize()
    dec.launch(d_file, n, b, s, 2)
    torch.cuda.synchronize()
    assert dec.stage_ms() == []
    assert_same_as_oracle(_arrays(b, dec.info(b)), want, "untimed")


def test_graph_capture_with_stage_timing_on():
    """Under stream capture the stage events (normally on the kernels' own dispatches) are recorded as graph nodes:
    capture works with timing on, replays give the oracle's records, and the captured events time the replay."""
    import torch

    from recordio import _lib as L
    from recordio import generate
    from recordio.device import DeviceDecoder, to_device_file

    img = generate(20_000, 1024, 2, kind=1, seed=41)
    dec = DeviceDecoder(0, own_ctx=True)
    d_file, n = to_device_file(img)
    b, _ = dec.decode(d_file, n, comp=2)
    assert L.lib().rio_ctx_set_timing(dec.ctx, 1) == L.RIO_OK
    g, s = _captured(dec, d_file, n, b, 2)
    _clear(b)
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        g.replay()
    torch.cuda.synchronize()
    assert_same_as_oracle(_arrays(b, dec.info(b)), orc.file_reader_decode_arrays(np.asarray(img)), "graph timed")
    ms = dec.stage_ms()
    assert len(ms) == 4 and all(x >= 0 for x in ms) and ms[3] > 0, ms


def test_reserve_covers_the_walk_flip_then_graph_capture(monkeypatch):
    """rio_ctx_reserve sizes the arenas for every walk the automatic choice can take: a context whose
    first decode takes the wave walk and whose hint then flips the next one to the lane walk (1 KiB records, lane
    chunks of 1 KiB here so 40 000 records fill the lane walk's chunk count) allocates nothing after the reserve,
    and that next call, captured into a HIP graph, replays to the oracle's records."""
    import torch

    from recordio import _lib as L
    from recordio import generate
    from recordio.device import DeviceDecoder, to_device_file

    monkeypatch.setenv("RIO_LANE_CHUNK_BYTES", "1024")
    img = generate(40_000, 1024, 0, kind=0, seed=31)
    dec = DeviceDecoder(0, own_ctx=True)  # the context reads RIO_LANE_CHUNK_BYTES at creation
    d_file, n = to_device_file(img)
    assert L.lib().rio_ctx_reserve(dec.ctx, n, 40_000, 1) == 0
    held = L.lib().rio_ctx_arena_bytes(dec.ctx)
    b = dec.alloc(40_000, 40_000 * 1024)
    s = torch.cuda.Stream(device=0)
    dec.launch(d_file, n, b, s, 0)  # fresh hint: the wave walk; its finalize writes ~1 036 bytes per record
    s.synchronize()
    assert L.lib().rio_ctx_arena_bytes(dec.ctx) == held
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        dec.launch(d_file, n, b, s, 0)  # the lane walk: 32 times the chunks, no allocation
    assert L.lib().rio_ctx_arena_bytes(dec.ctx) == held
    _clear(b)
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        g.replay()
    torch.cuda.synchronize()
    assert L.lib().rio_ctx_arena_bytes(dec.ctx) == held
    got = _arrays(b, dec.info(b))
    assert_same_as_oracle(got, orc.file_reader_decode_arrays(np.asarray(img)), "reserve + walk flip + graph")
