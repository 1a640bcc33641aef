"""Generates tests/golden/book_bgr.npz: the reference's data/book.jpg decoded
with PIL into imread's BGR byte order -- the input the front-end tests
(tests/test_frontend.py) convert; its gray conversion is the committed
book_gray.pgm.  Needs /root/reference (this container only).

    python tests/golden/make_frontend_golden.py
"""
import os

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
BOOK = "/root/reference/data/book.jpg"


def main():
    rgb = np.asarray(Image.open(BOOK).convert("RGB"), np.uint8)
    bgr = np.ascontiguousarray(rgb[..., ::-1])
    np.savez_compressed(os.path.join(HERE, "book_bgr.npz"), bgr=bgr)
    print(bgr.shape)


if __name__ == "__main__":
    main()
