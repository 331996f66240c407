"""Host logic of the directory driver (bitstream.use_model, utils.py:46-62): batching by shape
and pixel budget, file order, and the bounded PNG-writer queue -- with the device pass replaced
by a stub, so this runs on the CPU."""
import threading
import time

import numpy as np
import pytest
from PIL import Image

from neural_network_image_compression_amd import bitstream as B


class _Model:
    def load(self, path):
        self.loaded = path


@pytest.fixture
def dataset(tmp_path):
    d = tmp_path / "ds"
    d.mkdir()
    rng = np.random.default_rng(0)
    shapes = [(16, 24)] * 7 + [(8, 8)] * 3 + [(16, 24)] * 5
    for k, (h, w) in enumerate(shapes):
        Image.fromarray(rng.integers(0, 256, (h, w, 3), dtype=np.uint8)).save(d / f"{k:03d}.png")
    Image.fromarray(rng.integers(0, 256, (8, 8), dtype=np.uint8)).save(d / "grey.png")  # skipped (2-D)
    (d / "notes.txt").write_text("not an image")
    return d, shapes


def _stub(monkeypatch, log, delay):
    state = {"outstanding": 0, "max": 0}
    lock = threading.Lock()

    def job(names):
        time.sleep(delay)
        with lock:
            state["outstanding"] -= 1
        return names

    def feed_batch(model, x, filenames, output_dir, in_cshape, pool=None, png_threads=16):
        log.append((x.shape, list(filenames)))
        with lock:
            state["outstanding"] += 1
            state["max"] = max(state["max"], state["outstanding"])
        return [pool.submit(job, list(filenames))]

    monkeypatch.setattr(B, "feed_batch", feed_batch)
    return state


def test_writer_queue_is_bounded(tmp_path, dataset, monkeypatch):
    d, shapes = dataset
    log = []
    state = _stub(monkeypatch, log, delay=0.05)  # the writer is far slower than the "device"
    B.use_model(_Model(), str(d), "ckpt", str(tmp_path / "out"), 3, batch_size=2)
    assert state["max"] <= B.WRITES_IN_FLIGHT
    assert state["outstanding"] == 0  # every write finished before use_model returned
    names = [n for _, ns in log for n in ns]
    assert names == [f"{k:03d}" for k in range(len(shapes))]  # file order, grey image skipped
    assert all(len(ns) <= 2 for _, ns in log)
    for shape, ns in log:  # batches never mix shapes
        assert {shapes[int(n)] for n in ns} == {shape[1:3]}


def test_batch_pixel_budget(tmp_path, dataset, monkeypatch):
    d, _ = dataset
    log = []
    _stub(monkeypatch, log, delay=0.0)
    monkeypatch.setattr(B, "BATCH_PIXELS", 3 * 16 * 24)  # three 16 x 24 images per batch at most
    B.use_model(_Model(), str(d), "ckpt", str(tmp_path / "out"), 3, batch_size=64)
    for shape, _ in log:
        assert shape[0] * shape[1] * shape[2] <= B.BATCH_PIXELS
    assert [s[0] for s, _ in log] == [3, 3, 1, 3, 3, 2]


def test_write_error_is_raised(tmp_path, dataset, monkeypatch):
    d, _ = dataset

    def feed_batch(model, x, filenames, output_dir, in_cshape, pool=None, png_threads=16):
        def fail():
            raise OSError("disk full")
        return [pool.submit(fail)]

    monkeypatch.setattr(B, "feed_batch", feed_batch)
    with pytest.raises(OSError, match="disk full"):
        B.use_model(_Model(), str(d), "ckpt", str(tmp_path / "out"), 3)
