"""Face-tensor ingestion on the host side (no GPU): the oracle's OpenCV fixed-point restatement,
pinned by the reference's pickled gallery, and TheTrainer.read_images's walk / labels / decoding
(reference trainer/thetrainer.py:72-111) with a stub cv2 and with the PIL decoder."""
import os
import sys
import types

import numpy as np
import pytest

import facerec_oracle as O

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _gray_fixture():
    z = np.load(os.path.join(GOLDEN, "individuals_gray.npz"))
    off = np.concatenate([[0], np.cumsum(z["shapes"].prod(1))])
    imgs = [z["pixels"][off[i]:off[i + 1]].reshape(tuple(s)) for i, s in enumerate(z["shapes"])]
    return imgs, z["labels"], list(z["names"]), list(z["files"])


def test_oracle_resize_reproduces_pickled_gallery():
    """The reference's own training features (individuals.pkl, made with real cv2 by its authors) are
    reproduced from the bundled JPEGs through the restated INTER_LINEAR fixed point to < 2e-3
    (norm-relative), each by a gallery row of the right person -- the pin of the ingestion path."""
    imgs, labels, _, _ = _gray_fixture()
    m = np.load(os.path.join(GOLDEN, "individuals_model.npz"))
    W, G, gl = m["W"], m["gallery"], m["labels"]
    hit = set()
    for img, lab in zip(imgs, labels):
        q = O.cv_resize_u8(img, (70, 70), "linear").reshape(-1).astype(np.float64) @ W
        rel = np.linalg.norm(G - q, axis=1) / np.linalg.norm(q)
        j = int(np.argmin(rel))
        assert rel[j] < 2e-3 and gl[j] == lab, (rel[j], gl[j], lab)
        hit.add(j)
    assert len(hit) == 30          # 31 files, two byte-identical (steve_crop0 / steve_crop5)


@pytest.mark.parametrize("interp", ["linear", "cubic"])
def test_oracle_resize_properties(interp):
    r = np.random.default_rng(3)
    c = np.full((41, 67), 200, np.uint8)
    for size in [(70, 70), (13, 9), (134, 82)]:
        assert np.all(O.cv_resize_u8(c, size, interp) == 200)           # partition of unity (2048)
    img = r.integers(0, 256, (30, 44), dtype=np.uint8)
    assert np.array_equal(O.cv_resize_u8(img, (44, 30), interp), img)   # same size: copy
    up = O.cv_resize_u8(img, (88, 60), interp)
    assert up.shape == (60, 88) and up.dtype == np.uint8


def test_oracle_bgr2gray_weights():
    px = np.array([[[255, 0, 0], [0, 255, 0], [0, 0, 255], [255, 255, 255], [0, 0, 0]]], np.uint8)
    assert O.cv_bgr2gray(px).tolist() == [[29, 150, 76, 255, 0]]


def _dataset(tmp_path, imgs, files, writer):
    for img, f in zip(imgs, files):
        p = tmp_path / f
        p.parent.mkdir(parents=True, exist_ok=True)
        writer(p, img)
    (tmp_path / "empty_subject").mkdir()          # holds nothing: no label (thetrainer.py:94)
    return str(tmp_path)


def _expected(root, table):
    """thetrainer.py:87-110 restated on the test's own table: labels per non-empty folder in
    os.walk order, files in os.listdir order."""
    X, y, names, c = [], [], [], 0
    for dirname, dirnames, _ in os.walk(root):
        for sub in dirnames:
            sp = os.path.join(dirname, sub)
            if os.listdir(sp):
                names.append(sub)
                for f in os.listdir(sp):
                    X.append(table[f"{sub}/{f}"])
                    y.append(c)
                c += 1
    return X, y, names


def test_read_images_with_stub_cv2(tmp_path, monkeypatch):
    """cv2 importable (a stub whose imread serves the fixture's 70x70 faces): read_images is the
    reference's loop; no resize is needed at the faces' own size, so no device work happens."""
    faces = np.load(os.path.join(GOLDEN, "individuals_faces.npz"))
    files = [str(f).replace(".JPG", ".jpg") for f in faces["files"]]
    table = dict(zip(files, faces["X"]))
    root = _dataset(tmp_path, faces["X"], files, lambda p, img: p.write_bytes(b"stub"))
    stub = types.ModuleType("cv2")
    stub.IMREAD_GRAYSCALE = 0
    calls = []

    def imread(path, flag):
        calls.append(flag)
        rel = os.path.relpath(path, root)
        return table.get(rel)

    stub.imread = imread
    monkeypatch.setitem(sys.modules, "cv2", stub)
    from ocvfacerec.trainer.thetrainer import TheTrainer
    X, y, names = TheTrainer.read_images(root, (70, 70))
    eX, ey, enames = _expected(root, table)
    assert names == enames and y == ey and len(X) == 31
    assert all(np.array_equal(a, b) and a.dtype == np.uint8 for a, b in zip(X, eX))
    assert set(calls) == {0}
    assert sorted(set(y)) == [0, 1, 2, 3] and "empty_subject" not in names


def test_read_images_pil_decoder_without_cv2(tmp_path, monkeypatch):
    """No cv2: grey PNGs decode losslessly through PIL (image_size None: no resize)."""
    monkeypatch.setitem(sys.modules, "cv2", None)       # import cv2 -> ImportError
    from PIL import Image
    r = np.random.default_rng(5)
    imgs = [r.integers(0, 256, (20 + i, 30 - i), dtype=np.uint8) for i in range(6)]
    files = [f"p{i % 3}/img{i}.png" for i in range(6)]
    root = _dataset(tmp_path, imgs, files, lambda p, img: Image.fromarray(img, "L").save(p))
    from ocvfacerec.trainer.thetrainer import TheTrainer
    X, y, names = TheTrainer.read_images(root)
    eX, ey, enames = _expected(root, dict(zip(files, imgs)))
    assert names == enames and y == ey
    assert all(np.array_equal(a, b) for a, b in zip(X, eX))


def test_read_images_undecodable_file_raises(tmp_path, monkeypatch):
    """cv2.imread returns None for a non-image and the reference's next call raises
    (thetrainer.py:107-109): so does this one."""
    monkeypatch.setitem(sys.modules, "cv2", None)
    (tmp_path / "a").mkdir()
    (tmp_path / "a" / "notes.txt").write_text("not an image")
    from ocvfacerec.trainer.thetrainer import TheTrainer
    with pytest.raises(ValueError):
        TheTrainer.read_images(str(tmp_path))


def test_train_missing_dataset_exits(tmp_path):
    from ocvfacerec.trainer.thetrainer import TheTrainer
    with pytest.raises(SystemExit):
        TheTrainer(str(tmp_path / "nope"), (70, 70), str(tmp_path / "m.pkl")).train()
