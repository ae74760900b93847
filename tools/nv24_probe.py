"""Root-cause probe for the phased loss-head schedule above NV = 20.

Runs tests/test_grpo_edge_gpu.py::test_vocab_size_limits' case (T = 5 rows, V = 196 608 = 24 x 8192:
NV = 24) through the library named by PRL_LIB (default: the product build) and maps every dlogits
element that disagrees with the oracle onto the kernel's register layout: vector k (the lane's k-th
16-byte vector, buf[k]), lane (thread id in the 1024-thread workgroup), element j of the 8.
Also T = 600 (several rows per workgroup: the next-row loads of the phased schedule).
Prints one JSON line per case."""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests"), str(ROOT / "pipelinerl-swe_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import grpo_oracle, synth  # noqa: E402
from test_grpo_edge_gpu import CFG, _batch, _run  # noqa: E402


def main():
    V = int(os.environ.get("NV_PROBE_V", 196608))
    for T in (5, 600):
        b = _batch(T, V, seed=5)
        lg = synth.to_bf16(np.random.default_rng(5).normal(0, 2, (1, T, V))).astype(np.float32)
        loss, stats, d = _run(lg, b)
        o = grpo_oracle.rl_step_oracle(lg, b, CFG, 0, 10, dtype=np.float32, threads=16, row_chunk=8)
        want = o["dlogits"]
        err = np.abs(d - want)
        bad = err > (1e-8 + 1e-2 * np.abs(want))
        rows, cols = np.nonzero(bad[0])
        vec = cols // 8
        out = {"lib": os.environ.get("PRL_LIB", "product"), "T": T, "V": V, "bad": int(bad.sum()),
               "max_err": float(err.max()), "bad_rows": sorted(set(rows.tolist()))[:20],
               "bad_k": sorted(set((vec // 1024).tolist())), "bad_lanes_sample": sorted(set((vec % 1024).tolist()))[:16],
               "bad_j": sorted(set((cols % 8).tolist())),
               "loss_err": abs(loss - o["loss"]), "stat_loss": stats.get("loss"), "oracle_loss": o["stats"].get("loss")}
        if rows.size:
            r, c = int(rows[0]), int(cols[0])
            out["first_bad"] = {"row": r, "col": c, "got": float(d[0, r, c]), "want": float(want[0, r, c]),
                                "ratio_row": float(np.median(d[0, r][bad[0, r]] / np.where(want[0, r][bad[0, r]] == 0, np.nan,
                                                                                          want[0, r][bad[0, r]])))}
            wr = want[0, r]
            out["row_zero_got"] = bool(np.all(d[0, r] == 0))
            # where do the wrong values come from?  match each against this row's logits and the
            # oracle's gradient anywhere in the row (bf16-rounded), by column
            lg_r = lg[0, r]
            w_bf = synth.to_bf16(want[0, r].astype(np.float64)).astype(np.float32)
            cols_r = cols[rows == r]
            pairs = sorted({(int(c // 8) // 1024, int(c // 8) % 1024 % 64, int(c // 8) % 1024 // 64, int(c % 8))
                            for c in cols_r})
            out["bad_kind_count_row"] = len(cols_r)
            out["bad_wave_lane_row"] = sorted({(w, ln) for _, ln, w, _ in pairs})[:64]
            detail = []
            for c in cols_r[:24]:
                g = float(d[0, r, c])
                m_lg = np.nonzero(lg_r == g)[0]
                m_gr = np.nonzero(w_bf == np.float32(g))[0]
                detail.append({"col": int(c), "k": int(c // 8) // 1024, "tid": int(c // 8) % 1024, "j": int(c % 8),
                               "got": g, "want": float(want[0, r, c]), "logit": float(lg_r[c]),
                               "got_is_logit_at": [int(x) for x in m_lg[:4]], "got_is_grad_at": [int(x) for x in m_gr[:4]]})
            out["detail"] = detail
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
