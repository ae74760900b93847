"""Counter-based synthetic inputs (TEST INFRASTRUCTURE, shared by fixtures, tests and bench).

Deterministic without any RNG library state, so the GPU box can regenerate exactly the
inputs the golden fixtures were computed on (SURVEY.md §8(c) F2, §8(d) generator).

    h(seed, i)  = splitmix64((seed << 40) ^ i)                  (uint64, wrapping)
    u(seed, i)  = ((h >> 11) + 0.5) * 2^-53                      in (0, 1)
    n(seed, i)  = sqrt(-2 ln u(seed, 2i)) * cos(2 pi u(seed, 2i+1))
    logits[t,j] = sigma * n(seed, t*V + j)  (+ boost at column ids[t+1] when
                  u(seed ^ 0xABCD, t) < boost_frac)
    ids[t]      = h(seed + 1, t) mod id_range
"""

from __future__ import annotations

import numpy as np

_M = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(x: np.ndarray) -> np.ndarray:
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def h(seed: int, idx: np.ndarray) -> np.ndarray:
    base = np.uint64((int(seed) << 40) & 0xFFFFFFFFFFFFFFFF)
    return splitmix64(base ^ np.asarray(idx, dtype=np.uint64))


def uniform(seed: int, idx: np.ndarray) -> np.ndarray:
    return ((h(seed, idx) >> np.uint64(11)).astype(np.float64) + 0.5) * (2.0 ** -53)


def normal(seed: int, idx: np.ndarray) -> np.ndarray:
    idx = np.asarray(idx, dtype=np.uint64)
    u1 = uniform(seed, idx * np.uint64(2))
    u2 = uniform(seed, idx * np.uint64(2) + np.uint64(1))
    return np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * u2)


def token_ids(seed: int, T: int, id_range: int) -> np.ndarray:
    return (h(seed + 1, np.arange(T, dtype=np.uint64)) % np.uint64(id_range)).astype(np.int64)


def logits_rows(seed: int, rows: np.ndarray, V: int, ids: np.ndarray, sigma: float = 3.0,
                boost: float = 8.0, boost_frac: float = 0.7) -> np.ndarray:
    """float64 logits for the given row indices (row t predicts ids[t+1])."""
    rows = np.asarray(rows, dtype=np.int64)
    out = np.empty((rows.size, V), dtype=np.float64)
    cols = np.arange(V, dtype=np.uint64)
    bu = uniform(seed ^ 0xABCD, rows.astype(np.uint64))
    for k, t in enumerate(rows):
        out[k] = sigma * normal(seed, np.uint64(t) * np.uint64(V) + cols)
        if t + 1 < ids.size and bu[k] < boost_frac:
            out[k, ids[t + 1]] += boost
    return out


def to_bf16(x: np.ndarray) -> np.ndarray:
    """Round-to-nearest-even float -> bf16, returned as float32 values."""
    f = np.asarray(x, dtype=np.float32)
    u = f.view(np.uint32).astype(np.uint64)
    r = ((u + np.uint64(0x7FFF) + ((u >> np.uint64(16)) & np.uint64(1))) >> np.uint64(16)) << np.uint64(16)
    out = r.astype(np.uint32).view(np.float32)
    return np.where(np.isnan(f), f, out)


def bf16_bits(x: np.ndarray) -> np.ndarray:
    """bf16-exact float32 values -> uint16 bit patterns."""
    return (np.asarray(x, dtype=np.float32).view(np.uint32) >> 16).astype(np.uint16)


def packed_rl_batch(seed: int, seq_lens: list[int], prompt_lens: list[int], id_range: int,
                    eos: int | None = None, rewards: list[float] | None = None) -> dict:
    """A packed [1, T] batch in collate_packed layout (data.py:215-279).

    Per-token RL fields follow prepare_rl_fields / populate_rl_data
    (rl/__init__.py:504-525, 380-501): rewards constant per sequence, labels -100 on
    prompt tokens, old/ref log-probs 0 on prompt tokens, num_labels = #labels per sequence.
    old/ref log-probs for completion tokens are filled by the caller.
    """
    T = int(sum(seq_lens))
    ids = token_ids(seed, T, id_range)
    labels = ids.copy()
    pos = np.zeros(T, dtype=np.int64)
    rw = np.zeros(T, dtype=np.float32)
    adv = np.zeros(T, dtype=np.float32)
    gt = np.zeros(T, dtype=np.float32)
    nl = np.zeros(T, dtype=np.float32)
    ov = np.zeros(T, dtype=np.float32)
    bounds = [0]
    start = 0
    rnd = uniform(seed + 7, np.arange(len(seq_lens), dtype=np.uint64))
    for i, (n, p) in enumerate(zip(seq_lens, prompt_lens)):
        sl = slice(start, start + n)
        pos[sl] = np.arange(n)
        labels[start:start + p] = -100
        r = float(rewards[i]) if rewards is not None else float(rnd[i] > 0.5)
        rw[sl] = r
        nl[sl] = n - p
        gt[sl] = float(np.mean(seq_lens))
        if eos is not None:
            ov[sl] = 0.0 if eos in ids[sl] else 1.0
        start += n
        bounds.append(start)
    mean_r = float(np.mean([rw[b] for b in bounds[:-1]]))
    adv[:] = rw - mean_r
    return dict(input_ids=ids[None], labels=labels[None], attention_mask=np.ones((1, T), np.int64),
                position_ids=pos[None], rewards=rw[None], advantages=adv[None],
                ref_logprobs=np.zeros((1, T), np.float32), old_logprobs=np.zeros((1, T), np.float32),
                group_tokens=gt[None], num_labels=nl[None], overflow=ov[None],
                seq_boundaries=np.asarray(bounds, np.int32), is_packed=True, model_version=0)
