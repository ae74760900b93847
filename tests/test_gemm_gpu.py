"""prl_gemm (include/prl_gemm.h: the ROCm hipBLASLt through a C ABI) on MI355X: the three linear
passes and the fp32 accumulating weight gradient against fp32 GEMMs of the same bf16 operands,
ragged shapes, strided-free views, a tuned solution index, and the library it runs on."""

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _rand(shape, g, scale=1.0):
    return (torch.randn(shape, generator=g, device=DEV) * scale).to(torch.bfloat16)


def _close(got, ref, rtol=1e-2):
    err = float((got.float() - ref).abs().max())
    assert err <= rtol * float(ref.abs().max()) + 1e-6, err


def test_library_is_rocm_hipblaslt():
    from pipelinerl_amd import gemm

    s = gemm.library()
    assert "libhipblaslt.so" in s and "torch" not in s, s


@pytest.mark.parametrize("T,N,K", [(4096, 1536, 1536), (1000, 256, 1536), (37, 24, 8), (8192, 8960, 1536),
                                   (65536, 1536, 1536), (40000, 256, 1536)])
def test_linear_passes_match_fp32(T, N, K):
    from pipelinerl_amd import gemm

    g = torch.Generator(device=DEV).manual_seed(T + N + K)
    x, w, dy = _rand((T, K), g), _rand((N, K), g, 0.05), _rand((T, N), g)
    _close(gemm.linear_fwd(x, w), x.float() @ w.float().t())
    _close(gemm.linear_dgrad(dy, w), dy.float() @ w.float())
    _close(gemm.linear_wgrad(dy, x), dy.float().t() @ x.float())
    b = _rand((N,), g)
    _close(gemm.linear_fwd(x, w, b), x.float() @ w.float().t() + b.float())  # bias epilogue
    # leading batch dims are flattened like F.linear's
    y3 = gemm.linear_fwd(x.view(1, T, K), w)
    assert y3.shape == (1, T, N) and torch.equal(y3[0], gemm.linear_fwd(x, w))


def test_tuned_solutions_match_fp32():
    """Every swept solution in gemm_solutions.json, at its own token count, within bf16 rounding
    (checked on a row slice of the output for the big problems)."""
    from pipelinerl_amd import gemm

    for key, entries in sorted(gemm.solutions().items()):
        pas, N, K, dt, acc = key.split(":")
        N, K = int(N), int(K)
        for e in entries:
            T = e["T"]
            if e["index"] < 0:  # a routing entry (library heuristic): covered by the pass tests
                continue
            g = torch.Generator(device=DEV).manual_seed(T % 1000 + N)
            x, w = _rand((T, K), g), _rand((N, K), g, 0.05)
            if pas == "fwd":  # with and without the bias epilogue (q/k/v carry a bias)
                b = _rand((N,), g)
                y = gemm.linear_fwd(x, w, solution=e["index"])
                _close(y[:256], x[:256].float() @ w.float().t())
                y = gemm.linear_fwd(x, w, b, solution=e["index"])
                _close(y[:256], x[:256].float() @ w.float().t() + b.float())
            elif pas == "dgrad":
                dy = _rand((T, N), g)
                dx = gemm.linear_dgrad(dy, w)
                _close(dx[:256], dy[:256].float() @ w.float())
            else:
                dy = _rand((T, N), g)
                out = torch.zeros((N, K), device=DEV, dtype=torch.float32 if dt == "f32" else torch.bfloat16)
                gemm.linear_wgrad(dy, x, out=out, accumulate=acc == "1")
                ref = dy[:, :512].float().t() @ x.float()
                _close(out[:512], ref)
            del x, w
            torch.cuda.empty_cache()


def test_wgrad_fp32_accumulates_over_chunks():
    from pipelinerl_amd import gemm

    g = torch.Generator(device=DEV).manual_seed(3)
    V, H, T = 4096, 256, 3000
    h, dl = _rand((T, H), g), _rand((T, V), g)
    dw = torch.zeros((V, H), dtype=torch.float32, device=DEV)
    for a in range(0, T, 1024):  # ragged last chunk
        gemm.linear_wgrad(dl[a:a + 1024], h[a:a + 1024], out=dw, accumulate=True)
    ref = dl.double().t() @ h.double()
    assert float((dw.double() - ref).abs().max()) <= 1e-4 * float(ref.abs().max())


def test_solution_index_and_errors():
    from pipelinerl_amd import gemm

    lib = gemm.load()
    g = torch.Generator(device=DEV).manual_seed(9)
    T, N, K = 2048, 512, 256
    x, dy = _rand((T, K), g), _rand((T, N), g)
    idx = lib.prl_gemm_heuristic_index(0, 1, K, N, T, K, N, K, 1, 0.0)
    assert idx >= 0
    ref = gemm.linear_wgrad(dy, x)
    out = torch.empty_like(ref)
    shipped = sorted({int(e["index"]) for es in gemm.solutions().values() for e in es if int(e["index"]) >= 0})
    try:
        # an index outside the registered (swept) set is refused before any launch
        with pytest.raises(gemm.GemmError, match="allowed"):
            gemm.gemm(0, 1, K, N, T, x, K, dy, N, out, K, solution=idx if idx not in shipped else 10 ** 9)
        gemm.allow(shipped + [idx, 10 ** 9])
        gemm.gemm(0, 1, K, N, T, x, K, dy, N, out, K, solution=idx)  # the heuristic's own index
        assert torch.equal(out, ref)
        gemm.gemm(0, 1, K, N, T, x, K, dy, N, out, K, solution=10 ** 9)  # allowed, unknown: heuristic
        assert torch.equal(out, ref)
    finally:
        gemm.allow(shipped)
    with pytest.raises(gemm.GemmError):
        gemm.linear_wgrad(dy, x, out=torch.empty((N, K + 1), dtype=torch.bfloat16, device=DEV))
    with pytest.raises(gemm.GemmError):
        gemm.gemm(0, 0, K, N, T, x.float(), K, dy, N, out, K)


def test_streams_get_their_own_handles():
    """Each (device, stream) that issues a GEMM gets its own hipBLASLt handle and workspace (the
    gfx950 solutions are stream-K kernels: no launch may share fix-up state with another stream's,
    DESIGN.md §5).  The GEMMs here never overlap: each stream is drained before the next starts."""
    from pipelinerl_amd import gemm

    lib = gemm.load()
    g = torch.Generator(device=DEV).manual_seed(4)
    x = torch.randn((512, 384), generator=g, device=DEV).to(torch.bfloat16)
    w = torch.randn((640, 384), generator=g, device=DEV).to(torch.bfloat16)
    y0 = gemm.linear_fwd(x, w, solution=-1)
    torch.cuda.synchronize()
    n0 = lib.prl_gemm_handle_count()
    side = torch.cuda.Stream(device=DEV)
    with torch.cuda.stream(side):
        y1 = gemm.linear_fwd(x, w, solution=-1)
    side.synchronize()
    n1 = lib.prl_gemm_handle_count()
    with torch.cuda.stream(side):
        gemm.linear_fwd(x, w, solution=-1)
    side.synchronize()
    assert n1 == n0 + 1 and lib.prl_gemm_handle_count() == n1  # one more handle, reused after
    assert torch.equal(y0, y1)  # same plan choice on either handle
