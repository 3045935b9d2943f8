"""Device face-tensor ingestion (ofr_ingest_faces) and the restored trainer boundary.

* Bit-exact against the oracle's restatement of OpenCV's 8-bit fixed point (grey weights and
  INTER_LINEAR / INTER_CUBIC), on ragged batches of grey, BGR and BGRA images, crops, up- and
  down-scaling.  Parity with cv2 itself is unpinned (cv2 is absent); the pin is the reference's
  pickled gallery, reproduced from the bundled JPEGs through the device resize to < 2e-3.
* TheTrainer.train (trainer/thetrainer.py:142-179) end to end: a dataset folder read by
  read_images, computed, pickled; load_model's predictions equal train_arrays'.
* The recognizer path (bin/ocvf_recognizer.py:64-66): crops of BGR frames -> grey -> INTER_CUBIC
  on the device, predicted without a host round trip.
"""
import os
import sys
import types

import numpy as np
import pytest
import torch

import facerec_oracle as O

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    torch.cuda.set_device(0)


def _gray_fixture():
    z = np.load(os.path.join(GOLDEN, "individuals_gray.npz"))
    off = np.concatenate([[0], np.cumsum(z["shapes"].prod(1))])
    return [z["pixels"][off[i]:off[i + 1]].reshape(tuple(s)) for i, s in enumerate(z["shapes"])], z["labels"]


@pytest.mark.parametrize("interp", ["linear", "cubic"])
def test_ingest_bit_exact_vs_oracle(interp):
    from opencv_facerecognizer_amd import ingest
    r = np.random.default_rng(11 if interp == "linear" else 12)
    imgs = [r.integers(0, 256, (37, 53), dtype=np.uint8),                 # grey, up + down scaling
            r.integers(0, 256, (200, 161, 3), dtype=np.uint8),            # BGR, strong down-scaling
            r.integers(0, 256, (9, 14, 4), dtype=np.uint8),               # BGRA, strong up-scaling
            np.full((70, 70), 93, np.uint8),                              # same size: copy
            r.integers(0, 256, (480, 640, 3), dtype=np.uint8)]            # a camera frame (crops below)
    boxes = [(0, 0, 0, 53, 37), (1, 0, 0, 161, 200), (2, 0, 0, 14, 9), (3, 0, 0, 70, 70),
             (4, 100, 50, 260, 230), (4, 0, 0, 3, 2), (4, 637, 470, 640, 480), (1, 10, 20, 90, 21),
             (4, 0, 0, 640, 480)]                                          # whole frame: > 64 KiB of grey
    # (1100, 7): wider than the per-face kernel's tables -> the per-pixel kernel
    for size in [(70, 70), (23, 31), (100, 100), (1100, 7)]:
        got = ingest.faces(imgs, size, interp, boxes=boxes, host=True)
        for j, (i, x0, y0, x1, y1) in enumerate(boxes):
            crop = imgs[i][y0:y1, x0:x1]
            g = crop if crop.ndim == 2 else O.cv_bgr2gray(crop)
            ref = O.cv_resize_u8(g, size, interp)
            assert np.array_equal(got[j], ref), (size, j, np.abs(got[j].astype(int) - ref).max())


def test_ingest_rejects_bad_crops():
    from opencv_facerecognizer_amd import ingest
    with pytest.raises(ValueError):
        ingest.faces([np.zeros((10, 10), np.uint8)], (5, 5), boxes=[(0, 0, 0, 11, 5)])
    with pytest.raises(TypeError):
        ingest.faces([np.zeros((10, 10), np.float32)], (5, 5))
    assert ingest.faces([], (5, 5), host=True).shape == (0, 5, 5)


def test_ingest_reproduces_pickled_gallery():
    """The reference's pickled training features (made by its authors with real cv2) from the
    bundled JPEGs (libjpeg luma plane) through the DEVICE INTER_LINEAR resize, projected with the
    pickled W: every face within 2e-3 (norm-relative) of a gallery row of its own person."""
    from opencv_facerecognizer_amd import ingest
    from ocvfacerec.facerec.serialization import load_model
    imgs, labels = _gray_fixture()
    faces = ingest.faces(imgs, (70, 70), "linear")
    for i, im in enumerate(imgs):
        assert np.array_equal(faces[i].cpu().numpy(), O.cv_resize_u8(im, (70, 70), "linear"))
    model = load_model(os.path.join(GOLDEN, "individuals.pkl"))
    F = model.feature.project_device(faces, f64=True).cpu().numpy()
    G = np.stack([np.asarray(x).reshape(-1) for x in model.classifier.X])
    for f, lab in zip(F, labels):
        rel = np.linalg.norm(G - f, axis=1) / np.linalg.norm(f)
        j = int(np.argmin(rel))
        assert rel[j] < 2e-3 and model.classifier.y[j] == lab
    # and the model recognises every one of them from the device batch
    preds = model.predict_batch(faces)
    assert [p[0] for p in preds] == list(labels)


def test_trainer_train_roundtrip(tmp_path, monkeypatch):
    """TheTrainer.train on a folder dataset (cv2 stubbed: imread serves the full-size grey fixture,
    the resize to 70x70 runs on the device) writes a pickle that load_model reads back; its
    predictions equal those of train_arrays on the same faces."""
    from opencv_facerecognizer_amd import ingest
    from ocvfacerec.facerec.serialization import load_model
    from ocvfacerec.trainer.thetrainer import ExtendedPredictableModel, TheTrainer
    imgs, labels = _gray_fixture()
    z = np.load(os.path.join(GOLDEN, "individuals_gray.npz"))
    files = [str(f) for f in z["files"]]
    root = tmp_path / "data"
    table = {}
    for img, f in zip(imgs, files):
        p = root / f
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_bytes(b"stub")
        table[os.path.realpath(str(p))] = img
    stub = types.ModuleType("cv2")
    stub.IMREAD_GRAYSCALE = 0
    stub.imread = lambda path, flag: table.get(os.path.realpath(path))
    monkeypatch.setitem(sys.modules, "cv2", stub)
    out = str(tmp_path / "model.pkl")
    t = TheTrainer(str(root), (70, 70), out, None)
    X, y, names = t.read_images(str(root), (70, 70))
    assert sorted(names) == sorted(str(n) for n in z["names"])
    model = t.train()
    loaded = load_model(out)
    assert isinstance(loaded, ExtendedPredictableModel) and loaded.image_size == (70, 70)
    assert loaded.subject_names == dict(enumerate(names))
    ref = TheTrainer(None, (70, 70), str(tmp_path / "ref.pkl")).train_arrays(X, y, names)
    faces = ingest.faces(imgs, (70, 70), "linear")
    p1 = loaded.predict_batch(faces)
    p2 = ref.predict_batch(faces)
    p3 = model.predict_batch(faces)
    assert [a[0] for a in p1] == [b[0] for b in p2] == [c[0] for c in p3]
    for a, b in zip(p1, p2):
        assert np.allclose(a[1]["distances"], b[1]["distances"], rtol=1e-9)


def test_recognizer_frames_path():
    """bin/ocvf_recognizer.py:64-66 for several detections at once: crop + BGR2GRAY + INTER_CUBIC
    on the device, then predict_batch on the device faces == the same model on the oracle's faces."""
    from opencv_facerecognizer_amd import ingest
    from ocvfacerec.facerec.serialization import load_model
    model = load_model(os.path.join(GOLDEN, "individuals.pkl"))
    imgs, _ = _gray_fixture()
    r = np.random.default_rng(21)
    frames, boxes = [], []
    for i in (0, 9, 17, 26):                       # paste bundled faces into noisy BGR frames
        fr = r.integers(0, 256, (240, 320, 3), dtype=np.uint8)
        f = O.cv_resize_u8(imgs[i], (150, 150), "linear")
        fr[40:190, 60:210] = np.repeat(f[:, :, None], 3, axis=2)
        frames.append(fr)
        boxes.append((len(frames) - 1, 60, 40, 210, 190))
    dev = ingest.faces(frames, model.image_size, "cubic", boxes=boxes)
    host = [O.recognizer_face(frames[i], (x0, y0, x1, y1), model.image_size) for i, x0, y0, x1, y1 in boxes]
    assert np.array_equal(dev.cpu().numpy(), np.stack(host))
    got = model.predict_batch(dev)
    want = [model.predict(h) for h in host]
    assert [g[0] for g in got] == [w[0] for w in want]
    assert np.allclose([g[1]["distances"][0] for g in got], [w[1]["distances"][0] for w in want], rtol=1e-12)
