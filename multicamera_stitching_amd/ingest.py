"""Frame ingest either side of the stitch.

* DataReader: the reference's replay index (MediaPlayer/model.py data_reader, :51-128) -- the
  data.csv written by data_capture_node.py (:173-181, :296-307; header capture_id, timestamp,
  camera_label, image_file) parsed into images[capture][camera][timestamp] paths, timestamps per
  capture and the camera-label -> index map, with the same attribute names, quirks and summary
  text (tests/golden/ingest/ holds the reference's own parses).
* replay(): the video_mapping_node's LOCAL_RUN=2 loop (video_mapping_node.py:105-130): per
  step one images_dic in camera-label order, then the next timestamp, wrapping over captures;
  frames decoded (PIL; cv2.imread order BGR) by a pool of threads ahead of the consumer.
* concat_frame / StreamPipeline.submit_concat: the memmap bus layout (cameras side by side on
  axis 1, video_mapping_node.py:72-73, :140) fed to the pinned-staging stitch pipeline without
  splitting the frame first (mcs_stream_submit_strided gathers each camera's rows).
* ReplayStitcher: replay -> StreamPipeline (H2D / stitch / D2H overlapped) -> mosaics.
JPEG decoding stays on the host (no rocJPEG in this image); decoders differ in their IDCT, so a
mosaic matches the reference's bit for bit only for frames decoded by the same library.
"""
from __future__ import annotations

import csv
import os
from concurrent.futures import ThreadPoolExecutor
from collections import deque

import numpy as np


class DataReader:
    """images[i][j][k]: path of the image of capture i, camera j, timestamp k (model.py:3-9)."""

    def __init__(self):
        self.path = None
        self.timestamps = [[]]
        self.camera_labels = {}
        self.images = [[[]]]
        self.current_capture = None
        self.current_camera = None
        self.line_count = None
        self.header_format = None

    def __str__(self):
        lines = ["----DATA READER SUMMARY----\n", "Camera labels:", str(self.camera_labels)]
        text = "\n".join(lines) + "\n"
        for n, capture in enumerate(self.images):
            text += "\nCapture {}\n{} Cameras\n{} timestamps in total\n".format(
                n, len(capture), len(capture[0]))
        text += self.header_format
        text += "\n----Total lines read from the csv file: {} ----".format(self.line_count)
        return text

    def load_data(self, path):
        """Parses path/data.csv (model.py:51-122).  A camera row is placed by its position
        within its timestamp group; labels are taken from the first timestamp group only; a new
        capture id opens a new capture (ids are used as list indices, as in the reference)."""
        self.path = path
        cap = stamp = None
        labels_done = False
        first_group = True      # within the first timestamp group of the current capture
        cam = 0
        with open(os.path.join(path, "data.csv")) as f:
            for n, row in enumerate(csv.reader(f, delimiter=",")):
                if n == 0:
                    self.header_format = "\n----Column names are: {}----".format(" | ".join(row))
                    self.line_count = 1
                    continue
                c = int(row[0])
                if cap is None:
                    cap = c
                elif c != cap:
                    cap = c
                    self.images.append([[]])
                    self.timestamps.append([])
                    first_group = True
                    stamp = None
                if stamp is None or stamp != row[1]:
                    if stamp is not None:
                        labels_done = True
                        first_group = False
                    stamp = row[1]
                    self.timestamps[cap].append(stamp)
                    cam = 0
                elif first_group:
                    self.images[cap].append([])
                if not labels_done and row[2] not in self.camera_labels:
                    self.camera_labels[row[2]] = cam
                self.images[cap][cam].append(row[3])
                cam += 1
                self.line_count += 1
        self.current_capture = 0
        self.current_camera = len(self.camera_labels) - 1

    def get_image(self, timestamp_idx, camera_idx, capture_idx):
        return self.images[capture_idx][camera_idx][timestamp_idx]


def imread_bgr(path):
    """cv2.imread(path) for 8-bit colour images: H x W x 3 BGR u8, None when unreadable."""
    from PIL import Image
    try:
        with Image.open(path) as im:
            rgb = np.asarray(im.convert("RGB"))
    except (OSError, ValueError):
        return None
    return np.ascontiguousarray(rgb[..., ::-1])


def replay_order(reader, steps):
    """(capture, timestamp) of the first `steps` replay steps (video_mapping_node.py:123-128)."""
    cap = t = 0
    out = []
    for _ in range(steps):
        out.append((cap, t))
        if t < len(reader.timestamps[cap]) - 1:
            t += 1
        else:
            cap = cap + 1 if cap < len(reader.images) - 1 else 0
            t = 0
    return out


def replay(folder, steps, prefetch=8, threads=8, reader=None):
    """Yields `steps` images_dic (label -> BGR frame, None for unreadable files, as cv2.imread)
    in the node's replay order, decoding up to `prefetch` steps ahead on a thread pool."""
    reader = reader or DataReader()
    if reader.path is None:
        reader.load_data(folder)
    labels = list(reader.camera_labels.keys())
    order = replay_order(reader, steps)

    def load(ct):
        cap, t = ct
        return {lab: imread_bgr(os.path.join(folder, "data", reader.get_image(t, j, cap)))
                for j, lab in enumerate(labels)}

    with ThreadPoolExecutor(max_workers=threads) as pool:
        pending = deque()
        it = iter(order)
        for ct in it:
            pending.append(pool.submit(load, ct))
            if len(pending) >= prefetch:
                break
        while pending:
            yield pending.popleft().result()
            nxt = next(it, None)
            if nxt is not None:
                pending.append(pool.submit(load, nxt))


def concat_frame(images):
    """The memmap bus frame: cameras side by side on axis 1 (video_mapping_node.py:140)."""
    return np.concatenate(images, axis=1)


class ReplayStitcher:
    """replay() -> the plan's streaming pipeline -> mosaics, `depth` captures in flight.
    plan: a _capi.Plan whose camera order is `labels` (sorted, as Stitcher.img_labels)."""

    def __init__(self, plan, labels, depth=3, use_graphs=True):
        from . import _capi
        self.pipe = _capi.StreamPipeline(plan, depth, use_graphs)
        self.labels = list(labels)
        self.depth = depth

    def run(self, frames_iter):
        """frames_iter: images_dic per step.  Yields the mosaics in order (None for a step with
        an unreadable frame: the node skips those, :132-136)."""
        inflight = deque()
        for images_dic in frames_iter:
            cams = [images_dic.get(lab) for lab in self.labels]
            if any(c is None for c in cams):
                inflight.append(None)
            else:
                if sum(s is not None for s in inflight) >= self.depth:
                    while inflight and inflight[0] is None:
                        yield inflight.popleft()
                    yield self.pipe.wait(inflight.popleft())
                inflight.append(self.pipe.submit(cams))
        while inflight:
            s = inflight.popleft()
            yield None if s is None else self.pipe.wait(s)

    def close(self):
        self.pipe.close()
