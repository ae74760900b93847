"""Edge cases of the fused loss head on the GPU, each checked against the pinned oracle (or
the reference's own semantics where the oracle has no rows to compare)."""

import numpy as np
import pytest
import torch

from gpu_helpers import LogitsModel, rel_close, to_batch
from oracle import grpo_oracle, synth

pytestmark = pytest.mark.gpu
DEV = "cuda"
CFG = dict(policy_loss="ppo", kl_coef=0.05, final_kl_coef=0.05, entropy_bonus=0.01, final_entropy_bonus=0.01,
           epsilon=0.2, batch_size=3, clamp_log_ratio_ref_new_value=5)


def _batch(T, V, seed=0, lens=None, prompts=None):
    lens = lens or [T]
    prompts = prompts or [min(2, x - 1) for x in lens]
    b = synth.packed_rl_batch(seed, lens, prompts, id_range=V, eos=3)
    rng = np.random.default_rng(seed)
    m = b["labels"] != -100
    b["old_logprobs"] = np.where(m, rng.normal(-6, 1, (1, T)), 0).astype(np.float32)
    b["ref_logprobs"] = np.where(m, rng.normal(-6, 1, (1, T)), 0).astype(np.float32)
    return b


def _run(lg, b, cfg=CFG, dtype=torch.bfloat16, values=None, scale=1.0):
    from pipelinerl_amd.finetune.rl import RLConfig, rl_step

    model = LogitsModel(torch.tensor(lg, dtype=torch.float32).to(dtype).to(DEV),
                        None if values is None else torch.tensor(values, device=DEV))
    loss, stats = rl_step(model, to_batch(b), 0, 10, RLConfig(**cfg))
    (loss * scale).backward()
    torch.cuda.synchronize()
    return float(loss.detach()), stats, model.logits.grad.float().cpu().numpy()


def _cmp(lg, b, cfg=CFG, dtype=torch.bfloat16, values=None):
    loss, stats, d = _run(lg, b, cfg, dtype, values)
    o = grpo_oracle.rl_step_oracle(lg, b, cfg, 0, 10, values=values)
    for k, v in o["stats"].items():
        if np.isinf(v):
            assert stats[k] == v, (k, stats[k], v)
        else:
            assert abs(stats[k] - v) <= 1e-4 * max(1.0, abs(v)), (k, stats[k], v)
    tol = (1e-2, 1e-8) if dtype == torch.bfloat16 else (1e-4, 1e-7)
    ok, err = rel_close(d, o["dlogits"], *tol)
    assert ok, err
    return stats, d


def test_single_loss_row():
    T, V = 2, 512
    b = _batch(T, V, lens=[2], prompts=[1])
    lg = synth.to_bf16(np.random.default_rng(1).normal(0, 2, (1, T, V))).astype(np.float32)
    _cmp(lg, b)


def test_no_rows_and_sentinel_batch():
    from pipelinerl_amd.finetune.rl import RLConfig, rl_step
    from pipelinerl_amd.finetune.utils import create_sentinel_batch

    # L = 1: logits[:, :-1] is empty in the reference -> loss 0, stats {"input_size"}
    b = _batch(1, 64, lens=[1], prompts=[0])
    loss, stats, d = _run(np.zeros((1, 1, 64), np.float32), b)
    assert loss == 0.0 and stats == {"input_size": 1.0} and np.all(d == 0)
    # sentinel batch: all labels masked; the trainer multiplies the loss by 0
    sb = create_sentinel_batch(DEV, None, 0)
    model = LogitsModel(torch.randn(1, 8, 256, device=DEV, dtype=torch.bfloat16))
    loss, stats = rl_step(model, sb, 0, 10, RLConfig(**CFG))
    (loss * 0.0).backward()
    assert stats == {"input_size": 8.0}
    assert torch.count_nonzero(model.logits.grad) == 0


@pytest.mark.parametrize("scale", [1e-3, 30.0, 2000.0])
def test_extreme_magnitudes(scale):
    T, V = 17, 4096
    b = _batch(T, V, seed=2, lens=[9, 8], prompts=[2, 3])
    lg = synth.to_bf16(np.random.default_rng(2).normal(0, scale, (1, T, V))).astype(np.float32)
    _cmp(lg, b)


@pytest.mark.parametrize("temperature", [0.05, 3.0])
def test_temperature_extremes(temperature):
    T, V = 13, 2048
    b = _batch(T, V, seed=3)
    lg = synth.to_bf16(np.random.default_rng(3).normal(0, 3, (1, T, V))).astype(np.float32)
    _cmp(lg, b, dict(CFG, temperature=temperature))


def test_neg_inf_logits_off_target():
    """-inf logits (masked vocab entries): the reference's entropy is NaN for that row, the
    token loss is NaN (counted by num_nans) and nan_to_num drops it from the sums."""
    T, V = 9, 1024
    b = _batch(T, V, seed=4)
    lg = synth.to_bf16(np.random.default_rng(4).normal(0, 2, (1, T, V))).astype(np.float32)
    tgt = b["input_ids"][0, 1:]
    col = (tgt[3] + 1) % V
    lg[0, 3, col] = -np.inf
    loss, stats, d = _run(lg, b)
    o = grpo_oracle.rl_step_oracle(lg, b, CFG, 0, 10)
    assert stats["num_nans"] == o["stats"]["num_nans"] >= 1
    assert abs(loss - o["loss"]) <= 1e-4 * max(1, abs(o["loss"]))
    other = [r for r in range(T - 1) if r != 3]
    ok, err = rel_close(d[0, other], o["dlogits"][0, other], 1e-2, 1e-8)
    assert ok, err
    assert np.all(d[0, 3] == 0)  # non-finite token loss: no gradient (the reference gets NaN here)


@pytest.mark.parametrize("V", [24 * 8192, 24 * 8192 + 8, 24 * 8192 + 3])
def test_vocab_size_limits(V):
    """Largest register-resident vocab (NV = 24), the first streamed one, and a ragged one."""
    T = 5
    b = _batch(T, V, seed=5)
    lg = synth.to_bf16(np.random.default_rng(5).normal(0, 2, (1, T, V))).astype(np.float32)
    _cmp(lg, b)


def test_strided_logits_rows():
    """logits sliced out of a wider buffer (row stride > V) are consumed without a copy."""
    from pipelinerl_amd.finetune.rl import RLConfig, rl_step

    T, V, W = 11, 4096, 4096 + 64
    b = _batch(T, V, seed=6)
    full = synth.to_bf16(np.random.default_rng(6).normal(0, 2, (1, T, W))).astype(np.float32)
    base = torch.tensor(full).to(torch.bfloat16).to(DEV).requires_grad_(True)
    view = base[:, :, :V]
    assert view.stride(1) == W

    class M(torch.nn.Module):
        def forward(self, **kw):
            import types
            return types.SimpleNamespace(logits=view)

    loss, stats = rl_step(M(), to_batch(b), 0, 10, RLConfig(**CFG))
    loss.backward()
    o = grpo_oracle.rl_step_oracle(full[:, :, :V], b, CFG, 0, 10)
    for k, v in o["stats"].items():
        assert abs(stats[k] - v) <= 1e-4 * max(1.0, abs(v)), k
    g = base.grad.float().cpu().numpy()
    assert rel_close(g[:, :, :V], o["dlogits"], 1e-2, 1e-8)[0]
    assert np.all(g[:, :, V:] == 0)


def test_unpacked_bf16_value_head_ragged():
    """[B, L] padded batch (collate layout), bf16, value head, rows of different lengths."""
    B, L, V = 3, 16, 3000
    rng = np.random.default_rng(7)
    ids = rng.integers(0, V, (B, L))
    labels = ids.copy()
    lens = [16, 11, 6]
    for i, n in enumerate(lens):
        labels[i, :3] = -100
        labels[i, n:] = -100
    f = lambda v: np.asarray(v, np.float32)  # noqa: E731
    b = dict(input_ids=ids, labels=labels, attention_mask=np.ones((B, L), np.int64), is_packed=False,
             rewards=f(np.repeat([[1.0], [0.0], [1.0]], L, 1)), advantages=f(np.repeat([[0.3], [-0.6], [0.3]], L, 1)),
             ref_logprobs=f(rng.normal(-7, 1, (B, L))), old_logprobs=f(rng.normal(-7, 1, (B, L))),
             group_tokens=f(np.full((B, L), 11.0)), num_labels=f(np.repeat([[13.0], [8.0], [3.0]], L, 1)),
             overflow=f(np.zeros((B, L))))
    lg = synth.to_bf16(rng.normal(0, 2, (B, L, V))).astype(np.float32)
    values = f(rng.normal(0.2, 0.3, (B, L)))
    _cmp(lg, b, dict(CFG, value_loss_coef=0.1), values=values)


def test_multi_row_per_workgroup():
    """Qwen2.5's vocab (the resident kernel's NV = 19, read / write phased schedule) with ~2.3 rows
    per workgroup of the persistent grid, so rows with and without a next row are both taken (rows
    claimed from the workspace's counter): every row's dlogits and every statistic against the
    oracle, two runs bitwise identical."""
    V = 151936
    lens = [150, 200, 251]
    T = sum(lens)
    b = _batch(T, V, seed=9, lens=lens, prompts=[20, 30, 40])
    lg = synth.to_bf16(np.random.default_rng(9).normal(0, 2.5, (1, T, V))).astype(np.float32)
    stats1, d1 = _cmp(lg, b)
    _, stats2, d2 = _run(lg, b)
    assert np.array_equal(d1, d2) and stats2 == stats1


@pytest.mark.parametrize("V", [151936, 152064])
def test_resident_strided_rows_both_vocabularies(V):
    """Both Qwen2.5 vocabularies on the resident kernel, logits sliced out of a wider buffer (row
    stride V + 64)."""
    from pipelinerl_amd.finetune.rl import RLConfig, rl_step

    T, W = 9, V + 64
    b = _batch(T, V, seed=18)
    full = synth.to_bf16(np.random.default_rng(18).normal(0, 2, (1, T, W))).astype(np.float32)
    base = torch.tensor(full).to(torch.bfloat16).to(DEV).requires_grad_(True)
    view = base[:, :, :V]

    class M(torch.nn.Module):
        def forward(self, **kw):
            import types
            return types.SimpleNamespace(logits=view)

    loss, stats = rl_step(M(), to_batch(b), 0, 10, RLConfig(**CFG))
    loss.backward()
    o = grpo_oracle.rl_step_oracle(full[:, :, :V], b, CFG, 0, 10)
    for k, v in o["stats"].items():
        assert abs(stats[k] - v) <= 1e-4 * max(1.0, abs(v)), k
    g = base.grad.float().cpu().numpy()
    assert rel_close(g[:, :, :V], o["dlogits"], 1e-2, 1e-8)[0]
    assert np.all(g[:, :, V:] == 0)


@pytest.mark.parametrize("ent", [0.0, 0.01])
def test_target_columns_at_vector_edges(ent):
    """Targets on the edges of the register-resident row layout (Qwen2.5's V = 151 936: 19 vectors
    per lane, the last one partial): the target term is added by the owner lane after the row's
    stores (the phased schedule's fix-up), and entropy 0 takes the form without the entropy term."""
    T, V = 12, 151936
    b = _batch(T, V, seed=7, lens=[T], prompts=[1])
    cols = [0, 1, 7, 8, 8191, 8192, 147455, 147456, 147457, V - 8, V - 1]
    for r, col in enumerate(cols):
        b["input_ids"][0, 1 + r] = col
        if b["labels"][0, 1 + r] != -100:
            b["labels"][0, 1 + r] = col
    lg = synth.to_bf16(np.random.default_rng(7).normal(0, 2, (1, T, V))).astype(np.float32)
    cfg = dict(CFG, entropy_bonus=ent, final_entropy_bonus=ent)
    _, d = _cmp(lg, b, cfg)
    o = grpo_oracle.rl_step_oracle(lg, b, cfg, 0, 10)
    rows = [r for r in range(len(cols)) if b["labels"][0, 1 + r] != -100]
    assert len(rows) >= 8
    for r in rows:
        got, want = d[0, r, cols[r]], o["dlogits"][0, r, cols[r]]
        assert abs(got - want) <= 1e-2 * abs(want) + 1e-8, (r, cols[r], got, want)


# fp32 logits at a Qwen2.5 vocabulary take the pair kernel (grpo_fwd_pair_f32<19>: the row split
# over two workgroups, columns [0, 75 968) and [75 968, 151 936), each half in registers, 19 vectors
# per lane, the last one partial) or, with PrlGrpoParams.f32_rows = 1, the part-resident one
# (grpo_fwd_hybrid_f32<19, 9>: columns [0, 77 824) in registers, [77 824, 114 688) in LDS, the rest
# streamed and re-read).  pair_spin_ticks < 0: a half never waits for its partner — a partner whose
# claim or partial has not arrived yet at the first look sends the half SOLO (its own rows claimed,
# the other half's partial and gradient streamed from HBM: the bounded-spin path).
HYB_EDGES = [0, 3, 4, 77823, 77824, 77827, 114687, 114688, 114691, 151935]
PAIR_EDGES = [0, 3, 4, 73723, 73727, 73728, 75967, 75968, 75971, 75972, 149503, 149504, 151935]
F32_KERNELS = {"pair": {}, "pair_nowait": {"pair_spin_ticks": -1}, "hybrid": {"f32_rows": 1}}


def _controls(monkeypatch, **fields):
    """The loss head's kernel controls (PrlGrpoParams.pair_spin_ticks / f32_rows) for every launch
    rl_step makes while ``monkeypatch`` is active."""
    from pipelinerl_amd.finetune.rl.fused import GrpoParams

    orig = GrpoParams.to_c

    def to_c(self, write_grad):
        c = orig(self, write_grad)
        for k, v in fields.items():
            setattr(c, k, v)
        return c

    monkeypatch.setattr(GrpoParams, "to_c", to_c)


@pytest.fixture(params=list(F32_KERNELS))
def f32_kernel(request, monkeypatch):
    _controls(monkeypatch, **F32_KERNELS[request.param])
    return request.param


@pytest.mark.parametrize("ent", [0.0, 0.01])
def test_fp32_resident_targets_at_region_edges(ent, f32_kernel):
    """Targets on both sides of the half / vector boundaries (pair kernel) and of the register /
    LDS / streamed boundaries (hybrid), fp32 at 1e-4."""
    edges = HYB_EDGES if f32_kernel == "hybrid" else PAIR_EDGES
    T, V = len(edges) + 2, 151936
    b = _batch(T, V, seed=11, lens=[T], prompts=[1])
    for r, col in enumerate(edges):
        b["input_ids"][0, 1 + r] = col
        if b["labels"][0, 1 + r] != -100:
            b["labels"][0, 1 + r] = col
    lg = np.random.default_rng(11).normal(0, 2, (1, T, V)).astype(np.float32)
    cfg = dict(CFG, entropy_bonus=ent, final_entropy_bonus=ent)
    _, d = _cmp(lg, b, cfg, dtype=torch.float32)
    o = grpo_oracle.rl_step_oracle(lg, b, cfg, 0, 10)
    for r, col in enumerate(edges):
        if b["labels"][0, 1 + r] != -100:
            assert rel_close(d[0, r, col], o["dlogits"][0, r, col], 1e-4, 1e-7)[0], col


def test_fp32_resident_many_rows_per_workgroup_and_non_finite(f32_kernel, monkeypatch):
    """~2.3 rows per workgroup pair (hybrid: per workgroup) — rows with and without a successor,
    slots / the LDS slab reused row after row —, a -inf in each half of one row each; two runs
    bitwise identical (for the pair kernel also against the run that never waits: the partner's
    partial computed from HBM is the same bits as the one it publishes)."""
    V = 151936
    lens = [150, 200, 251]
    T = sum(lens)
    b = _batch(T, V, seed=12, lens=lens, prompts=[20, 30, 40])
    lg = np.random.default_rng(12).normal(0, 2.5, (1, T, V)).astype(np.float32)
    tgt = b["input_ids"][0, 1:]
    for r, col in ((40, 140000), (41, 30000)):
        lg[0, r, col if col != tgt[r] else col + 1] = -np.inf
    loss, stats, d1 = _run(lg, b, dtype=torch.float32)
    o = grpo_oracle.rl_step_oracle(lg, b, CFG, 0, 10)
    assert stats["num_nans"] == o["stats"]["num_nans"] >= 2
    assert abs(loss - o["loss"]) <= 1e-4 * max(1, abs(o["loss"]))
    other = [r for r in range(T - 1) if r not in (40, 41)]
    ok, err = rel_close(d1[0, other], o["dlogits"][0, other], 1e-4, 1e-7)
    assert ok, err
    assert np.all(d1[0, [40, 41]] == 0)
    _, _, d2 = _run(lg, b, dtype=torch.float32)
    assert np.array_equal(d1, d2)
    if f32_kernel == "pair":
        with monkeypatch.context() as m:
            _controls(m, pair_spin_ticks=-1)
            loss3, stats3, d3 = _run(lg, b, dtype=torch.float32)
        assert np.array_equal(d1, d3) and loss3 == loss and stats3 == stats


def test_fp32_resident_strided_rows(f32_kernel):
    """fp32 logits sliced out of a wider buffer (row stride V + 64) at a Qwen2.5 vocabulary."""
    from pipelinerl_amd.finetune.rl import RLConfig, rl_step

    T, V, W = 9, 151936, 151936 + 64
    b = _batch(T, V, seed=13)
    full = np.random.default_rng(13).normal(0, 2, (1, T, W)).astype(np.float32)
    base = torch.tensor(full).to(DEV).requires_grad_(True)
    view = base[:, :, :V]
    assert view.stride(1) == W

    class M(torch.nn.Module):
        def forward(self, **kw):
            import types
            return types.SimpleNamespace(logits=view)

    loss, stats = rl_step(M(), to_batch(b), 0, 10, RLConfig(**CFG))
    loss.backward()
    o = grpo_oracle.rl_step_oracle(full[:, :, :V], b, CFG, 0, 10)
    for k, v in o["stats"].items():
        assert abs(stats[k] - v) <= 1e-4 * max(1.0, abs(v)), k
    g = base.grad.cpu().numpy()
    assert rel_close(g[:, :, :V], o["dlogits"], 1e-4, 1e-7)[0]
    assert np.all(g[:, :, V:] == 0)


@pytest.mark.parametrize("V", [65536, 65536 + 4, 114688, 152064, 196608])
def test_fp32_pair_kernel_vocab_range(V):
    """Vocabularies across the pair kernel's range (half rows of 8 .. 19 vectors per lane; odd
    vector counts give halves of different lengths) and one past it (196 608: the hybrid kernel),
    a few rows each, fp32 at 1e-4."""
    T = 6
    b = _batch(T, V, seed=14)
    lg = np.random.default_rng(14).normal(0, 2, (1, T, V)).astype(np.float32)
    _cmp(lg, b, dtype=torch.float32)


@pytest.mark.parametrize("dtype,env", [(torch.float32, {})], ids=["fp32_pair"])
def test_pair_kernels_beside_a_kernel_holding_cus(dtype, env, monkeypatch):
    """The fp32 pair kernel beside a long kernel on another stream that holds registers on half the CUs
    (as an RCCL collective beside the loss head would): half the workgroups start only as others
    finish; a half whose partner is late stops waiting after the (lowered, 20 us) spin bound and
    computes the partner's partial itself.  The launch completes with the same bits as the
    uncontended run's (which matches the oracle), and prl_grpo_pair_fallbacks counts the halves
    that did not wait."""
    import ctypes

    from pipelinerl_amd import _native
    from pipelinerl_amd.finetune.rl import RLConfig, rl_step

    for k, v in env.items():
        monkeypatch.setenv(k, v)
    V = 151936
    lens = [200, 200]
    T = sum(lens)
    b = _batch(T, V, seed=19, lens=lens, prompts=[20, 20])
    lg = np.random.default_rng(19).normal(0, 2, (1, T, V)).astype(np.float32)
    if dtype == torch.bfloat16:
        lg = synth.to_bf16(lg).astype(np.float32)
    loss0, stats0, d0 = _run(lg, b, dtype=dtype)
    o = grpo_oracle.rl_step_oracle(lg, b, CFG, 0, 10)
    tol = (1e-2, 1e-8) if dtype == torch.bfloat16 else (1e-4, 1e-7)
    assert rel_close(d0, o["dlogits"], *tol)[0]

    lib = _native.load()
    fallbacks = _fallbacks_reader(lib)
    fallbacks()
    hog = torch.empty(1 << 30, dtype=torch.uint8, device=DEV)
    sink = torch.zeros(256, dtype=torch.int32, device=DEV)
    side = torch.cuda.Stream()
    _controls(monkeypatch, pair_spin_ticks=2000)  # 20 us
    model = LogitsModel(torch.tensor(lg, dtype=torch.float32).to(dtype).to(DEV))
    torch.cuda.synchronize()
    with torch.cuda.stream(side):  # ~50 ms of 128 workgroups reading 1 GiB at 20 GB/s
        assert lib.prl_paced_read(ctypes.c_void_p(hog.data_ptr()), hog.numel(), 20.0, 128,
                                  ctypes.c_void_p(sink.data_ptr()), side.cuda_stream) == 0
    loss, stats = rl_step(model, to_batch(b), 0, 10, RLConfig(**CFG))
    loss.backward()
    torch.cuda.synchronize()
    d1 = model.logits.grad.float().cpu().numpy()
    assert np.array_equal(d0, d1)
    assert float(loss.detach()) == loss0 and stats == stats0
    # pairs are blocks b, b ^ 8 of 16-block groups: dispatched in order onto the free CUs, both halves
    # of a pair mostly start together, so the counter is usually 0 here (the never-wait runs of
    # test_*_many_rows_* go SOLO); it must be readable and bounded (a row is finished SOLO at most
    # once by each half)
    assert 0 <= fallbacks() <= 2 * (T - 1)
    # the counter counts: in the never-wait arm partners go SOLO at their first look
    _controls(monkeypatch, pair_spin_ticks=-1)
    _run(lg, b, dtype=dtype)
    assert fallbacks() > 0


def _fallbacks_reader(lib):
    """prl_grpo_pair_fallbacks on the current stream's workspace (fused._workspace): read and reset."""
    import ctypes

    from pipelinerl_amd.finetune.rl.fused import _workspace

    def fallbacks() -> int:
        ws = _workspace(torch.device(DEV))
        n = ctypes.c_uint64(0)
        assert lib.prl_grpo_pair_fallbacks(ctypes.c_void_p(ws.data_ptr()), ws.numel(),
                                           ctypes.c_void_p(torch.cuda.current_stream().cuda_stream),
                                           ctypes.byref(n)) == 0
        return int(n.value)

    return fallbacks


def test_pair_halves_far_apart_wait_once_not_every_row():
    """The fp32 pair kernel's waits are bounded per launch, not per row (halves that
    drift two or more rows apart used to wait the full 200 us spin on every remaining row, 64 rows x
    200 us = 12.8 ms per half here).  8 192 rows (64 per pair) run beside a long GEMM on a side stream
    that competes for the CUs: the launch costs about the GEMM's hold plus the rows, results
    bit-identical to the uncontended launch (measured on MI355X: 2.15 ms alone, 3.89 ms beside a
    2.34 ms GEMM, no fallback — the GEMM's tiles delay both halves of a pair alike).  Then a 10 ns
    spin bound (pair_spin_ticks 1): halves time out on their first late partner and go SOLO for the
    rest of the launch (their own rows claimed, the other half's partial and gradient from HBM) —
    the same bits."""
    import dataclasses

    from pipelinerl_amd import _native
    from pipelinerl_amd.finetune.rl.fused import GrpoParams, grpo_loss, prepare_fields

    lib = _native.load()
    V, T = 151936, 8193
    b = _batch(T, V, seed=23, lens=[4097, 4096], prompts=[1, 1])
    lg = torch.randn((1, T, V), generator=torch.Generator(device=DEV).manual_seed(23), device=DEV) * 2
    fields = prepare_fields(to_batch(b), DEV)
    params = GrpoParams(policy_loss="ppo", epsilon=0.2, kl_coef=0.05, entropy_coef=0.0, clamp_log_ratio=5.0,
                        temperature=1.0, batch_size=4.0)
    fallbacks = _fallbacks_reader(lib)

    def launch():
        x = lg.detach().requires_grad_(True)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        loss, stats, rows = grpo_loss(x, fields, params)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1), rows.clone(), stats.clone()

    launch()
    t0, rows0, stats0 = launch()
    fallbacks()
    ga = torch.randn((2048, 131072), device=DEV, dtype=torch.bfloat16)
    gb = torch.randn((131072, 4096), device=DEV, dtype=torch.bfloat16)
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        torch.mm(ga, gb)  # warm the GEMM's kernel selection
    torch.cuda.synchronize()
    es0, es1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(side):
        es0.record(side)
        torch.mm(ga, gb)
        es1.record(side)
    t1, rows1, stats1 = launch()
    torch.cuda.synchronize()
    hold = es0.elapsed_time(es1)
    fb = fallbacks()
    print(f"uncontended {t0:.2f} ms, beside the {hold:.2f} ms hold {t1:.2f} ms, fallbacks {fb}")
    assert torch.equal(rows0, rows1) and torch.equal(stats0, stats1)
    assert t1 <= hold + 3 * t0 + 2.0, (t0, t1, hold, fb)
    params1 = dataclasses.replace(params, pair_spin_ticks=1)
    x = lg.detach().requires_grad_(True)
    loss2, stats2, rows2 = grpo_loss(x, fields, params1)
    torch.cuda.synchronize()
    fb2 = fallbacks()
    print(f"spin bound 10 ns: fallbacks {fb2} of {2 * (T - 1)} row halves")
    assert torch.equal(rows0, rows2) and torch.equal(stats0, stats2)


def test_pair_claimed_rows_beside_side_workgroups():
    """The fp32 pair kernel claims its rows (round 6): beside 16 long-running side workgroups (an
    RCCL collective's channels: prl_paced_read, 1 GiB at 20 GB/s, ~50 ms) the pairs on the CUs they
    share take fewer rows instead of a static share, so the launch stays near its uncontended time
    (static rows: 13.2 -> 23.0 ms per C2 launch beside 16 side workgroups, claimed: 12.6 -> 13.7 ms,
    bench.py loss_head_fp32.beside_16_side_workgroups) — with the same bits and no SOLO rows."""
    import ctypes

    from pipelinerl_amd import _native
    from pipelinerl_amd.finetune.rl.fused import GrpoParams, grpo_loss, prepare_fields

    lib = _native.load()
    V, T = 151936, 16385
    b = _batch(T, V, seed=29, lens=[8193, 8192], prompts=[1, 1])
    lg = torch.randn((1, T, V), generator=torch.Generator(device=DEV).manual_seed(29), device=DEV) * 2
    fields = prepare_fields(to_batch(b), DEV)
    params = GrpoParams(policy_loss="ppo", epsilon=0.2, kl_coef=0.05, entropy_coef=0.0, clamp_log_ratio=5.0,
                        temperature=1.0, batch_size=4.0)
    fallbacks = _fallbacks_reader(lib)
    hog = torch.empty(1 << 30, dtype=torch.uint8, device=DEV)
    sink = torch.zeros(16, dtype=torch.int32, device=DEV)
    side = torch.cuda.Stream()

    def launch(beside: bool):
        x = lg.detach().requires_grad_(True)
        torch.cuda.synchronize()
        if beside:
            with torch.cuda.stream(side):
                assert lib.prl_paced_read(ctypes.c_void_p(hog.data_ptr()), hog.numel(), 20.0, 16,
                                          ctypes.c_void_p(sink.data_ptr()), side.cuda_stream) == 0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        loss, stats, rows = grpo_loss(x, fields, params)
        e1.record()
        torch.cuda.synchronize()
        loss.backward()
        return e0.elapsed_time(e1), rows.clone(), stats.clone(), x.grad

    launch(False)
    t0, rows0, stats0, g0 = launch(False)
    fallbacks()
    times = []
    for _ in range(3):
        t1, rows1, stats1, g1 = launch(True)
        times.append(t1)
        assert torch.equal(rows0, rows1) and torch.equal(stats0, stats1) and torch.equal(g0, g1)
        del g1
    fb = fallbacks()
    t1 = sorted(times)[1]
    print(f"uncontended {t0:.2f} ms, beside 16 side workgroups {times} ms, SOLO rows {fb}")
    assert t1 <= 1.35 * t0 + 0.3, (t0, times)


def test_claimed_rows_on_concurrent_streams():
    """Two loss-head launches in flight at once on two streams (each workgroup claims rows from its
    stream's own counter, grpo_loss.hip launch_resident_rows): both results equal the same launches
    run one after the other."""
    from pipelinerl_amd.finetune.rl.fused import GrpoParams, grpo_loss, prepare_fields

    V = 151936
    params = GrpoParams(policy_loss="ppo", epsilon=0.2, kl_coef=0.05, entropy_coef=0.0, clamp_log_ratio=5.0,
                        temperature=1.0, batch_size=4.0)
    runs = []
    for seed in (21, 22):
        lens = [900, 1100]
        b = _batch(sum(lens), V, seed=seed, lens=lens, prompts=[30, 40])
        lg = torch.tensor(synth.to_bf16(np.random.default_rng(seed).normal(0, 2.5, (1, sum(lens), V))),
                          dtype=torch.float32).to(torch.bfloat16).to(DEV)
        runs.append((lg, prepare_fields(to_batch(b), DEV)))

    def launch(lg, fields):
        x = lg.detach().clone().requires_grad_(True)
        loss, stats, rows = grpo_loss(x, fields, params)
        loss.backward()
        return x.grad, stats, rows

    seq = [launch(*r) for r in runs]
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    out = [None, None]
    for i, (st, r) in enumerate(zip((s1, s2), runs)):
        st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(st):
            out[i] = launch(*r)
    torch.cuda.synchronize()
    for a, b in zip(seq, out):
        for x, y in zip(a, b):
            assert torch.equal(x, y)
