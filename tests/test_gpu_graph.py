"""Stream capture: the library's calls are stream-ordered launches with no
host synchronisation once a device's constant tables exist, so a caller can
capture them into a HIP graph (here through torch.cuda.graph, which captures
the current stream) and replay the whole render + STFT of a file with one
launch -- what an application rendering many short files repeatedly wants.
Replays must give the eager call's bits, and follow new input contents.
"""
import numpy as np
import pytest

import dspbench as d

pytestmark = pytest.mark.gpu


def _eager_and_graph(torch, fn, x):
    """fn(x) -> tensors: eager results, then a captured graph's replay on
    the same input and on a changed one (compared with eager on that)."""
    want = [t.clone() for t in fn(x)]          # eager; also creates the device tables
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):              # warm the capture stream's scratch
        fn(x)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):     # capture on the warmed stream
        outs = fn(x)
    g.replay()
    torch.cuda.synchronize()
    for a, b in zip(outs, want):
        assert torch.equal(a, b)
    x.mul_(-0.5)                               # new contents, same buffer
    want2 = [t.clone() for t in fn(x)]
    g.replay()
    torch.cuda.synchronize()
    for a, b in zip(outs, want2):
        assert torch.equal(a, b)
    return outs


@pytest.mark.parametrize("plugin", ["gain_test", "IR_test", "no_op"])
@pytest.mark.parametrize("B", [512, 384])
def test_render_stft_captured(torch_cuda, plugin, B):
    torch = torch_cuda
    mk = {"gain_test": lambda: d.Plugin.gain_test(0.7), "IR_test": lambda: d.Plugin.ir_test(0.9, 0.002),
          "no_op": lambda: d.Plugin.no_op()}[plugin]
    L = 8192 * 7 + 300
    x = torch.from_numpy(np.random.default_rng(B).uniform(-1, 1, (2, L)).astype(np.float32)).cuda()
    nb = d.num_blocks(L, B)
    out = torch.empty((2, nb * B), device="cuda")
    mag = torch.empty((2, d.stft_frames(nb * B, 8192, 4096), 4097), device="cuda")
    p = mk()

    def fn(xx):
        return d.render_stft(xx, 2, B, 48000.0, p, out=out, mag=mag)
    _eager_and_graph(torch, fn, x)


def test_stft_and_render_chain_captured(torch_cuda):
    """Two calls in one graph: a render, then the STFT of another signal."""
    torch = torch_cuda
    L = 8192 * 5
    x = torch.from_numpy(np.random.default_rng(7).uniform(-1, 1, (2, L)).astype(np.float32)).cuda()
    out = torch.empty((2, L), device="cuda")
    mag = torch.empty((2, d.stft_frames(L, 8192, 4096), 4097), device="cuda")
    p = d.Plugin.gain_test(0.25)

    def fn(xx):
        r = d.render_offline(xx, 2, 512, 48000.0, p, out=out)
        m = d.stft_magnitude(xx, out=mag)
        return r, m
    _eager_and_graph(torch, fn, x)


def test_capture_on_a_cold_stream_is_refused_cleanly(torch_cuda):
    """A shape that needs per-stream scratch, captured on a stream that never
    ran it eagerly: a clear DSP_ERR_INVALID, not an allocation inside the
    capture (IR_test with a step whose ramp is not closed-form, B = 384)."""
    torch = torch_cuda
    L = 8192 * 3
    x = torch.zeros((2, L), device="cuda")
    p = d.Plugin.ir_test(0.8, 0.0013)
    d.render_stft(x, 2, 384, 48000.0, p)      # device tables exist
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with pytest.raises(Exception) as e:
        with torch.cuda.graph(g, stream=side):
            d.render_stft(x, 2, 384, 48000.0, p)
    assert "eager call" in str(e.value) or "capture" in str(e.value)
    torch.cuda.synchronize()
