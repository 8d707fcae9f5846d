#!/usr/bin/env python3
"""BF Hamming kNN-2 (mcs_match_hamming_knn2) throughput: pairs/s and VALU
utilisation (the matcher is VALU popcount-bound, so it is priced against the
vector integer rate, not HBM).

Per (query, train) pair the algorithm needs 8 v_xor_b32 + 8 accumulating v_bcnt_u32_b32 (the
256-bit Hamming distance): 16 integer lane-ops.  Peak = 256 CUs x 4 SIMDs x 32 lanes x 2.4 GHz
= 78.6 T lane-ops/s (MI355X_MICROARCH.md: a wave64 VALU op issues over 2 cycles on a SIMD-32), so
`popcount_util` = 16 * pairs/s / 78.6e12.  Timed with HIP events on the stream the kernels are
enqueued on (memset + kNN-2 + finalize per call); checked against the CPU restatement
(oracle/orc_match.c) at the smallest size.  One JSON line.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PEAK_LANE_OPS = 256 * 4 * 32 * 2.4e9
OPS_PER_PAIR = 16


def main():
    import torch
    from multicamera_stitching_amd import _capi
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream()
    rng = np.random.default_rng(0)
    lines = []
    for n in (2000, 8000, 32000):
        qh = rng.integers(0, 256, (n, 32), dtype=np.uint8)
        th = rng.integers(0, 256, (n, 32), dtype=np.uint8)
        q, t = torch.from_numpy(qh).to(dev), torch.from_numpy(th).to(dev)
        idx = torch.empty((n, 2), dtype=torch.int32, device=dev)
        dist = torch.empty((n, 2), dtype=torch.int32, device=dev)

        def call():
            _capi.match_hamming_knn2_device(q.data_ptr(), n, t.data_ptr(), n, idx.data_ptr(),
                                            dist.data_ptr(), 0, s.cuda_stream)
        for _ in range(3):
            call()
        reps = max(5, int(2e10 / (n * n)))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(s)
        for _ in range(reps):
            call()
        e1.record(s)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        pairs = n * n / (ms * 1e-3)
        line = {"n_query": n, "n_train": n, "ms_per_call": round(ms, 4),
                "pairs_per_s": float("%.4g" % pairs),
                "popcount_util": round(OPS_PER_PAIR * pairs / PEAK_LANE_OPS, 4), "reps": reps}
        if n == 2000:
            from oracle import oracle
            wi, wd = oracle.hamming_knn2(qh, th)
            line["max_abs_diff_vs_cpu"] = int(max(np.abs(idx.cpu().numpy() - wi).max(),
                                                  np.abs(dist.cpu().numpy() - wd).max()))
        lines.append(line)
    print(json.dumps({"metric": "BF Hamming kNN-2 pairs/s (256-bit descriptors)",
                      "unit": "pairs/s", "peak_lane_ops_per_s": PEAK_LANE_OPS,
                      "ops_per_pair": OPS_PER_PAIR, "sizes": lines}))


if __name__ == "__main__":
    main()
