"""Fixture for the ingestion tests: the 31 bundled face JPEGs of the reference
(/root/reference/data/individuals/<name>/*.jpg) decoded to grey at full size.

Decoding = libjpeg's grayscale output (PIL ``draft('L')``), which is what
``cv2.imread(path, cv2.IMREAD_GRAYSCALE)`` asks libjpeg for (trainer/thetrainer.py:99).
The resize to 70x70 is NOT applied here: tests/test_gpu_ingest.py runs it on the device.
Writes tests/golden/individuals_gray.npz: pixels (concatenated), shapes [31][2], labels,
names, files -- in the label order of individuals.pkl (dennis, linus, bill, steve).
Run in the build container (needs /root/reference); the npz is committed.
"""
import os

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = "/root/reference/data/individuals"
NAMES = ["dennis", "linus", "bill", "steve"]


def main():
    pix, shapes, labels, files = [], [], [], []
    for c, nm in enumerate(NAMES):
        for f in sorted(os.listdir(os.path.join(ROOT, nm))):
            with Image.open(os.path.join(ROOT, nm, f)) as im:
                im.draft("L", im.size)
                g = np.asarray(im.convert("L"), dtype=np.uint8)
            pix.append(g.reshape(-1))
            shapes.append(g.shape)
            labels.append(c)
            files.append(f"{nm}/{f}")
    np.savez_compressed(os.path.join(HERE, "individuals_gray.npz"), pixels=np.concatenate(pix),
                        shapes=np.asarray(shapes, np.int64), labels=np.asarray(labels, np.int64),
                        names=np.asarray(NAMES), files=np.asarray(files))


if __name__ == "__main__":
    main()
