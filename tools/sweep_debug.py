"""Debug aid (tools only): one blended stitch vs the C restatement, with the multi-band sweep and
with the band pass + blend (MCS_MB_SWEEP=0); prints where they differ and saves the arrays."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle import oracle  # noqa: E402
from test_gpu_blend import _world_plan  # noqa: E402

CASES = {
    "c0": dict(n=4, w=320, h=180, ch=3, seed=3),
    "c1": dict(n=3, w=200, h=120, ch=1, seed=4, rot_deg=4.0, persp=1e-4),
    "c4": dict(n=3, w=180, h=100, ch=3, seed=7, super_mode=True, rot_deg=3.0),
    "big": dict(n=4, w=1920, h=1080, ch=3, seed=0),
}


def run(name, sweep):
    os.environ["MCS_MB_SWEEP"] = "1" if sweep else "0"
    case = dict(CASES[name])
    interp = case.pop("interp", 1)
    plan, cams = _world_plan(interp=interp, **case)
    plan.set_blend(2)
    got = plan.stitch_host(cams)
    st = plan.stats()
    want, owner = oracle.blend_stitch(plan.describe(), cams, 2, interp, want_owner=True)
    got = got.reshape(want.shape)
    d = np.abs(got.astype(np.int16) - want.astype(np.int16))
    if d.ndim == 3:
        d = d.max(2)
    ys, xs = np.nonzero(d)
    print(f"{name} sweep={sweep} stats={ {k: v for k, v in st.items() if k.startswith('mb')} } max={int(d.max())} n_bad={len(ys)}")
    if len(ys):
        print("  bad rows", ys.min(), ys.max(), "cols", xs.min(), xs.max())
        for y, x in list(zip(ys, xs))[:12]:
            print(f"   ({y},{x}) got {got[y, x]} want {want[y, x]} owner {owner[y, x]}")
        np.savez_compressed(f"gpurun_out/sweep_dbg_{name}.npz", got=got, want=want, owner=owner)


if __name__ == "__main__":
    for name in sys.argv[1:] or ["c0"]:
        run(name, True)
        run(name, False)
