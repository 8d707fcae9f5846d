"""Debug helper (round 4): runs the C2 full-size multi-band device stitch several times, compares
the runs with each other and with the oracle, and prints where they differ (blend tiles,
owners, values)."""
import sys

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from test_gpu_blend import _world_plan  # noqa: E402
from oracle import oracle  # noqa: E402


def main():
    import torch
    plan, cams = _world_plan(4, 1920, 1080, 3, seed=0)
    plan.set_blend(2)
    F = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    shots = [[np.roll(c, 7 * f, axis=0) for c in cams] for f in range(F)]
    dev = [torch.from_numpy(np.stack([shots[f][i] for f in range(F)])).cuda()
           for i in range(len(cams))]
    want = [oracle.blend_stitch(plan.describe(), shots[f], 2) for f in range(F)]
    outs = []
    for rep in range(4):
        out = torch.zeros((F, plan.out_h, plan.out_w * 3), dtype=torch.uint8, device="cuda")
        plan.stitch_device([d.data_ptr() for d in dev], [d[0].numel() for d in dev],
                           out.data_ptr(), plan.out_w * 3, out[0].numel(), F, 0)
        torch.cuda.synchronize()
        got = out.cpu().numpy().reshape(F, plan.out_h, plan.out_w, 3)
        outs.append(got)
        for f in range(F):
            d = np.abs(got[f].astype(int) - want[f].astype(int)).max(axis=-1)
            ys, xs = np.nonzero(d)
            print(f"rep {rep} capture {f}: {len(ys)} px differ, max {d.max()}", end="")
            if len(ys):
                ty, tx = ys // 64, xs // 32
                tiles = sorted(set(zip(ty.tolist(), tx.tolist())))
                print(f", blend tiles (row, col) {tiles[:12]}{' ...' if len(tiles) > 12 else ''};"
                      f" rows {ys.min()}-{ys.max()} cols {xs.min()}-{xs.max()}")
            else:
                print()
    for rep in range(1, 4):
        print("rep", rep, "== rep 0:", bool(np.array_equal(outs[rep], outs[0])))
    print(plan.stats())


if __name__ == "__main__":
    main()
