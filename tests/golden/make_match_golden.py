"""Generates tests/golden/match.npz: knnMatch (k = 2) results of the CPU
restatement oracle/match.py on real SIFT descriptors from the committed
fixtures (book.npz, synth1_240x320.npz), so the GPU matcher is pinned to
fixed vectors and the oracle against regressions.

    python tests/golden/make_match_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import match as M  # noqa: E402


def main():
    book = np.load(os.path.join(HERE, "book.npz"), allow_pickle=False)["desc"]
    synth = np.load(os.path.join(HERE, "synth1_240x320.npz"), allow_pickle=False)["desc"]
    rng = np.random.default_rng(7)
    # a train set with exact duplicates and a perturbed copy of the queries:
    # equal distances (tie order) and near-ties both occur
    dup = np.concatenate([synth[:40], book[rng.permutation(len(book))[:64]], synth[:40]])
    noisy = (book + rng.normal(0, 1e-3, book.shape).astype(np.float32)).astype(np.float32)
    out = {}
    for name, q, t in [("book_synth", book, synth), ("synth_book", synth, book),
                       ("book_dup", book, dup), ("book_noisy", book, noisy)]:
        idx, dist = M.knn_match(q, t, 2)
        out[f"{name}_idx"], out[f"{name}_dist"] = idx, dist
    out["noisy"] = noisy
    out["dup"] = dup
    np.savez_compressed(os.path.join(HERE, "match.npz"), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
