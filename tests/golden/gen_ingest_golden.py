"""Generates tests/golden/ingest/*: synthetic data.csv files in the format the reference's
data_capture_node writes (data_capture_node.py:173-181, 296-307: header capture_id, timestamp,
camera_label, image_file; one row per camera per timestamp) and the parse the reference's own
MediaPlayer/model.py data_reader makes of them (run from /root/reference at generation time;
model.py imports only csv).  The fixtures are data: csv inputs + JSON outputs."""
import importlib.util
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "ingest")
REF = "/root/reference/MediaPlayer/model.py"

CASES = {
    # 1 capture, 3 timestamps, 4 cameras
    "one_capture": [(0, 1000 + 33 * t, lab, f"ab{t:02d}-{1000 + 33 * t}_{lab}.jpg")
                    for t in range(3) for lab in ["CAM1", "CAM2", "CAM3", "CAM4"]],
    # 3 captures with 2 / 4 / 1 timestamps, labels not in sorted order
    "three_captures": [(c, 5000 * (c + 1) + 40 * t, lab, f"cd-{c}-{t}_{lab}.jpg")
                       for c, nt in enumerate([2, 4, 1]) for t in range(nt)
                       for lab in ["LEFT", "CENTER", "RIGHT"]],
    # a single camera
    "single_camera": [(0, 10 + t, "CAM0", f"x{t}.jpg") for t in range(5)],
    # header only
    "empty": [],
}


def main():
    spec = importlib.util.spec_from_file_location("ref_model", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    for name, rows in CASES.items():
        d = os.path.join(OUT, name)
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "data.csv"), "w") as f:
            f.write("capture_id,timestamp,camera_label,image_file\n")
            for r in rows:
                f.write(",".join(str(v) for v in r) + "\n")
        dr = mod.data_reader()
        try:
            dr.load_data(d)
            res = dict(ok=True, images=dr.images, timestamps=dr.timestamps,
                       camera_labels=list(dr.camera_labels.items()), line_count=dr.line_count,
                       header_format=dr.header_format, current_capture=dr.current_capture,
                       current_camera=dr.current_camera, summary=str(dr))
        except Exception as e:     # the reference's own failure mode on this input
            res = dict(ok=False, error=type(e).__name__)
        with open(os.path.join(d, "expected.json"), "w") as f:
            json.dump(res, f, indent=1, sort_keys=True)
        print(name, "ok" if res["ok"] else res["error"])


if __name__ == "__main__":
    sys.exit(main())
