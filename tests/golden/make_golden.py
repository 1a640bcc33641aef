"""Generate the committed golden fixtures under tests/golden/.

Run from the repo root:  python tests/golden/make_golden.py   (--8k, --batch: the
large-size digest sets)

What is made, and from what:
  book_gray.pgm   data/book.jpg of the reference, decoded with PIL and converted
                  exactly as the reference's readImage does (src/main.cpp:79-86:
                  imread -> BGR bytes, cvtColor(COLOR_RGB2GRAY) on BGR data, i.e.
                  Y = (4899*B + 9617*G + 1868*R + 8192) >> 14, then CV_32FC1).
                  The JPEG decoder (PIL/libjpeg-turbo vs OpenCV's libjpeg) is not
                  the reference's, so the pixels are unpinned against it; the
                  fixture fixes them for every later comparison.
  *.npz           outputs of the CPU oracle (oracle/sift_oracle.c) on those
                  inputs: keypoints (cv::KeyPoint records), descriptors, and
                  SHA-256 digests of every Gaussian / DoG plane.

PARITY UNPINNED: the reference itself cannot be built in this image (OpenCV
4.0 + contrib absent) and ships no golden vectors, so these are regression
vectors of the restatement, not reference outputs.  Only data is stored
(numpy arrays, np.load(allow_pickle=False)).
"""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")
BOOK = "/root/reference/data/book.jpg"


def write_pgm(path, img_u8):
    h, w = img_u8.shape
    with open(path, "wb") as f:
        f.write(b"P5\n%d %d\n255\n" % (w, h))
        f.write(img_u8.astype(np.uint8).tobytes())


def read_pgm(path):
    with open(path, "rb") as f:
        data = f.read()
    parts = data.split(maxsplit=4)
    assert parts[0] == b"P5"
    w, h, mx = int(parts[1]), int(parts[2]), int(parts[3])
    assert mx == 255
    return np.frombuffer(parts[4][:w * h], np.uint8).reshape(h, w)


def book_gray():
    from PIL import Image
    rgb = np.asarray(Image.open(BOOK).convert("RGB")).astype(np.int64)
    R, G, B = rgb[..., 0], rgb[..., 1], rgb[..., 2]
    # imread gives B,G,R channel order; COLOR_RGB2GRAY weights channel 0 as R.
    return ((4899 * B + 9617 * G + 1868 * R + 8192) >> 14).astype(np.uint8)


def digests(packed, rows, cols, n_oct, per):
    return np.array([hashlib.sha256(p.tobytes()).hexdigest()
                     for p in O.split_planes(packed, rows, cols, n_oct, per)])


def case(name, img, with_planes=True, store_full=True):
    img = np.ascontiguousarray(img, np.float32)
    r, c = img.shape
    g = O.build_gaussian_pyramid(img, 5)
    d = O.build_dog_pyramid(g, r, c, 5)
    kps, desc = O.sift(img, 5)
    out = dict(rows=r, cols=c, n=len(kps),
               kp_sha=hashlib.sha256(kps.tobytes()).hexdigest(),
               desc_sha=hashlib.sha256(desc.tobytes()).hexdigest())
    if with_planes:
        out["gpyr_sha"] = digests(g, r, c, 5, 5)
        out["dog_sha"] = digests(d, r, c, 5, 4)
    if store_full:
        out["kps"] = kps.view(np.uint8).reshape(len(kps), 28) if len(kps) else np.zeros((0, 28), np.uint8)
        out["desc"] = desc
    np.savez_compressed(os.path.join(OUT, name + ".npz"), **out)
    print(f"{name}: {r}x{c} -> {len(kps)} keypoints")


def batch_1080():
    """configs[2] / configs[1] check vectors: seeds 0, 31, 63 of the bench's
    64-image 1080p batch (image b of bench.py's rank 0 is seed b), and seed
    0 with 4 octaves (configs[1]), defined as the 5-octave output filtered to
    octave <= 3 ('Config mismatch')."""
    seeds = [0, 31, 63]
    out = dict(seeds=np.array(seeds), rows=1080, cols=1920)
    n, ks, ds = [], [], []
    for b in seeds:
        kps, desc = O.sift(O.synth_image(b, 1080, 1920), 5)
        n.append(len(kps))
        ks.append(hashlib.sha256(kps.tobytes()).hexdigest())
        ds.append(hashlib.sha256(desc.tobytes()).hexdigest())
        if b == 0:
            keep = (kps["octave"] & 255) <= 3
            out["oct4_n"] = int(keep.sum())
            out["oct4_kp_sha"] = hashlib.sha256(kps[keep].tobytes()).hexdigest()
            out["oct4_desc_sha"] = hashlib.sha256(np.ascontiguousarray(desc[keep]).tobytes()).hexdigest()
        print(f"batch seed {b}: {len(kps)} keypoints")
    out.update(n=np.array(n), kp_sha=np.array(ks), desc_sha=np.array(ds))
    np.savez_compressed(os.path.join(OUT, "batch_1080x1920.npz"), **out)


def main():
    O.build()
    if "--batch" in sys.argv:
        batch_1080()
        return
    if "--8k" in sys.argv:
        # configs[4]: one 7680x4320 image (digests only; about 2 minutes of CPU)
        O.set_threads(os.cpu_count() or 1)
        case("synth0_4320x7680", O.synth_image(0, 4320, 7680), store_full=False)
        return
    if os.path.exists(BOOK):
        write_pgm(os.path.join(OUT, "book_gray.pgm"), book_gray())
    book = read_pgm(os.path.join(OUT, "book_gray.pgm")).astype(np.float32)
    case("book", book)
    case("synth0_160x128", O.synth_image(0, 160, 128))
    case("synth1_240x320", O.synth_image(1, 240, 320))
    case("synth2_203x157", O.synth_image(2, 203, 157))
    if "--no-1080" not in sys.argv:
        case("synth0_1080x1920", O.synth_image(0, 1080, 1920), store_full=False)


if __name__ == "__main__":
    main()
