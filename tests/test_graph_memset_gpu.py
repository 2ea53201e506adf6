"""Standalone HIP-graph capture checks for ``hipMemsetAsync``.

Round 3 replaced the zero fill in front of the accumulating split-K reduce (store-mode gradients,
csrc/elementwise.hip ``jm_zero_f32``) with a kernel because a step captured with the memset left
garbage in those gradients on replay.  These tests isolate the memset node from the framework:
the same call (``hipMemsetAsync(ptr, 0, bytes, current stream)``, issued here through ctypes on
the stream torch captures) is captured between a kernel that dirties the range and a kernel that
accumulates into it, over the shapes, offsets and sizes of the real gradients, and the replayed
result must equal eager execution.  Each case also runs the kernel replacement the framework
uses now.  Results and reading: profiles/r4_graph_memset.txt.
"""

import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu


def _hip():
    for name in ("libamdhip64.so", "libamdhip64.so.7", "libamdhip64.so.6"):
        try:
            return ctypes.CDLL(name)
        except OSError:
            continue
    pytest.skip("libamdhip64 not loadable")


def _memset(hip, t: torch.Tensor):
    st = torch.cuda.current_stream().cuda_stream
    rc = hip.hipMemsetAsync(ctypes.c_void_p(t.data_ptr()), ctypes.c_int(0), ctypes.c_size_t(t.numel() * t.element_size()),
                            ctypes.c_void_p(st))
    assert rc == 0, rc


# (flat elements, offset of the gradient view, view elements): ViT-L FF / QKV kernel gradients, a
# jumbo slice, an odd offset and a size that is not a multiple of 64
CASES = [(1 << 24, 4096, 4096 * 1024), (1 << 24, 123 * 64, 3072 * 1024), (1 << 23, 64, 12288 * 256),
         (1 << 22, 17, 1000 * 33), (1 << 20, 0, 4100)]


# Round 4 measurement (profiles/r4_graph_memset.txt): the captured memset reproduces the round-3
# failure on its own -- the first replay is right, later ones leave garbage in the range -- while
# the zero-fill kernel is exact on every replay.  The memset cases document the platform behaviour
# (xfail, not strict: a fixed runtime turns them into XPASS); the framework never captures a memset.
MEMSET_XFAIL = pytest.mark.xfail(reason="hipMemsetAsync captured in a HIP graph: wrong on replay (ROCm 7.x)",
                                 strict=False)


@pytest.mark.parametrize("total,off,n", CASES)
@pytest.mark.parametrize("how", [pytest.param("memset", marks=MEMSET_XFAIL), "kernel"])
def test_captured_zero_then_accumulate(total, off, n, how):
    hip = _hip()
    from jumbo_mae_tpu_amd.ops import _ext
    ext = _ext.load(True)
    flat = torch.full((total,), 3.0, device="cuda")
    g = flat[off:off + n]
    part = torch.arange(n, device="cuda", dtype=torch.float32).remainder_(97.0)
    before, after = flat[:off], flat[off + n:]

    def step():
        g.fill_(-5.0)  # last step's values (a store-mode gradient is not zeroed by zero_grad)
        if how == "memset":
            _memset(hip, g)
        else:
            ext.zero_f32(g)
        g.add_(part)  # the accumulating reduce

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()  # warmup on the side stream (torch's capture recipe)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    assert torch.equal(g, part)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        step()
    for rep in range(20):
        flat.fill_(3.0)
        flat[off:off + n].fill_(float(rep))
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(g, part), (how, rep, (g - part).abs().max().item())
        assert bool((before == 3.0).all()) and bool((after == 3.0).all()), "write outside the view"


@pytest.mark.parametrize("n", [4100, 1 << 16, 4096 * 1024])
def test_captured_memset_alone_diagnostic(n):
    """The memset node alone (no kernel around it): record which replays leave the range non-zero and
    what the bytes look like (written to gpurun_out/graph_memset_diag.txt for the profile record).
    Never fails: it characterises the runtime, the xfail cases above state the expectation."""
    import os
    hip = _hip()
    buf = torch.full((n + 64,), 7.0, device="cuda")
    g = buf[32:32 + n]
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        _memset(hip, g)
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        _memset(hip, g)
    lines = []
    for rep in range(4):
        buf.fill_(7.0)
        graph.replay()
        torch.cuda.synchronize()
        bad = (g != 0).nonzero().flatten()
        guard = bool((buf[:32] == 7.0).all()) and bool((buf[32 + n:] == 7.0).all())
        first = bad[:4].tolist()
        bits = [hex(int(v)) for v in g.view(torch.int32)[bad[:4]].tolist()] if len(bad) else []
        lines.append(f"n={n} replay={rep} nonzero={len(bad)} first={first} bits={bits} guards_ok={guard}")
    root = os.environ.get("GRAFT_REPO_ROOT", os.getcwd())
    os.makedirs(os.path.join(root, "gpurun_out"), exist_ok=True)
    with open(os.path.join(root, "gpurun_out", "graph_memset_diag.txt"), "a") as f:
        f.write("\n".join(lines) + "\n")
