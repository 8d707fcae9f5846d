"""Frame ingest on the CPU: the replay index against the reference's own
data_reader parses (tests/golden/ingest/, made by gen_ingest_golden.py from
MediaPlayer/model.py), the node's replay order, BGR decoding, the bus layout."""
import json
import os

import numpy as np
import pytest

from multicamera_stitching_amd import ingest

GOLD = os.path.join(os.path.dirname(__file__), "golden", "ingest")
CASES = sorted(d for d in os.listdir(GOLD) if os.path.isdir(os.path.join(GOLD, d)))


@pytest.mark.parametrize("case", CASES)
def test_data_reader_matches_reference_parse(case):
    want = json.load(open(os.path.join(GOLD, case, "expected.json")))
    r = ingest.DataReader()
    r.load_data(os.path.join(GOLD, case))
    assert want["ok"]
    assert r.images == want["images"]
    assert r.timestamps == want["timestamps"]
    assert list(r.camera_labels.items()) == [tuple(p) for p in want["camera_labels"]]
    assert r.line_count == want["line_count"]
    assert r.header_format == want["header_format"]
    assert (r.current_capture, r.current_camera) == (want["current_capture"],
                                                     want["current_camera"])
    assert str(r) == want["summary"]


def test_replay_order_wraps_like_the_node():
    r = ingest.DataReader()
    r.load_data(os.path.join(GOLD, "three_captures"))
    got = ingest.replay_order(r, 9)
    assert got == [(0, 0), (0, 1), (1, 0), (1, 1), (1, 2), (1, 3), (2, 0), (0, 0), (0, 1)]


def test_replay_decodes_bgr_in_label_order(tmp_path):
    from PIL import Image
    rng = np.random.default_rng(0)
    labels = ["CAM2", "CAM1"]
    os.makedirs(tmp_path / "data")
    rows = ["capture_id,timestamp,camera_label,image_file"]
    frames = {}
    for t in range(3):
        for lab in labels:
            img = rng.integers(0, 256, (12, 20, 3), dtype=np.uint8)      # RGB on disk
            name = f"p-{t}_{lab}.png"
            Image.fromarray(img).save(tmp_path / "data" / name)
            frames[(t, lab)] = img[..., ::-1]                            # cv2.imread: BGR
            rows.append(f"0,{100 + t},{lab},{name}")
    rows.append(f"0,200,CAM2,missing.png")
    rows.append(f"0,200,CAM1,p-0_CAM1.png")
    (tmp_path / "data.csv").write_text("\n".join(rows) + "\n")
    out = list(ingest.replay(str(tmp_path), 5, prefetch=2, threads=2))
    for t in range(3):
        assert list(out[t].keys()) == labels
        for lab in labels:
            assert np.array_equal(out[t][lab], frames[(t, lab)])
    assert out[3]["CAM2"] is None and np.array_equal(out[3]["CAM1"], frames[(0, "CAM1")])
    assert np.array_equal(out[4]["CAM2"], frames[(0, "CAM2")])           # wrapped around


def test_concat_frame_is_the_bus_layout():
    a = np.zeros((4, 5, 3), np.uint8)
    b = np.ones((4, 7, 3), np.uint8)
    f = ingest.concat_frame([a, b])
    assert f.shape == (4, 12, 3) and (f[:, 5:] == 1).all() and (f[:, :5] == 0).all()
