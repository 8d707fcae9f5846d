"""Ingest on the GPU: the memmap bus layout straight into the streaming
pipeline, and a data.csv + JPEG replay stitched end to end, bit-exact against the CPU
restatement of the same decoded frames."""
import os

import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu


def _rig(n=4, w=320, h=180, seed=0):
    from multicamera_stitching_amd import rig
    st, images, _ = rig.calibrated_stitcher(n, w, h, 3, seed=seed, rot_deg=1.5)
    stages = [dict(H=np.asarray(sb.cachedAH), canvas_w=sb.ABSize[0], canvas_h=sb.ABSize[1],
                   bx=sb.Bpts[0][0], by=sb.Bpts[0][1], super_mode=sb.super_mode,
                   x_limits=sb.x_limits, y_limits=sb.y_limits) for sb in st.stitchers]
    return st, images, stages


def test_submit_concat_equals_dense_submit():
    from multicamera_stitching_amd import _capi, ingest
    st, images, stages = _rig()
    cams = [images[label] for label in st.img_labels]
    sp = _capi.StreamPipeline(st.plan(), 2, True)
    try:
        frame = ingest.concat_frame(cams)
        a = sp.wait(sp.submit_concat(frame))
        b = sp.wait(sp.submit(cams))
        # a strided view (every other row of a taller buffer) works too
        tall = np.repeat(frame, 2, axis=0)[::2]
        c = sp.wait(sp.submit_concat(tall))
    finally:
        sp.close()
    want = oracle.cascade_stitch(stages, cams)
    for got in (a, b, c):
        assert np.array_equal(got.reshape(want.shape), want)


def test_csv_jpeg_replay_stitched_end_to_end(tmp_path):
    from PIL import Image
    from multicamera_stitching_amd import ingest
    st, images, stages = _rig(seed=2)
    labels = list(st.img_labels)
    os.makedirs(tmp_path / "data")
    rows = ["capture_id,timestamp,camera_label,image_file"]
    for t in range(6):
        for lab in labels:
            img = np.roll(images[lab], 3 * t, axis=1)[..., ::-1]            # BGR -> RGB file
            name = f"ab-{1000 + t}_{lab}.jpg"
            Image.fromarray(img).save(tmp_path / "data" / name, quality=80)
            rows.append(f"0,{1000 + t},{lab},{name}")
    (tmp_path / "data.csv").write_text("\n".join(rows) + "\n")
    rs = ingest.ReplayStitcher(st.plan(), labels, depth=3)
    try:
        got = list(rs.run(ingest.replay(str(tmp_path), 8, prefetch=4, threads=4)))
    finally:
        rs.close()
    assert len(got) == 8
    for step, mosaic in enumerate(got):
        t = step % 6
        cams = [ingest.imread_bgr(str(tmp_path / "data" / f"ab-{1000 + t}_{lab}.jpg"))
                for lab in labels]
        want = oracle.cascade_stitch(stages, cams)
        assert np.array_equal(mosaic.reshape(want.shape), want), step
