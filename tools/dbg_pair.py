"""Debug: fast pyramid (pyramid_pair) plane 0 of octave 1 vs the decimation
of the kernel's own octave-0 plane 3."""
import os, sys
import numpy as np
import torch  # noqa
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sift-gpu_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import siftgpu, oracle
for shape in ((1080, 1920), (203, 157), (300, 210)):
    img = oracle.synth_image(0, *shape)
    c = siftgpu.Context(*shape, 1, device=0, flags=1)
    gp = c.buildGaussianPyramid(img, 5)
    c.close()
    p3, b1 = gp[3], gp[5]
    dec = p3[0::2, 0::2][:b1.shape[0], :b1.shape[1]]
    d = np.abs(dec - b1)
    bad = np.argwhere(d > 1e-6)
    print(shape, "max", d.max(), "nbad", len(bad), "first", bad[:5].tolist(), "rows bad", np.unique(bad[:, 0])[:20].tolist() if len(bad) else [],
          "cols bad", np.unique(bad[:, 1])[:20].tolist() if len(bad) else [])
    if len(bad):
        r, cc = bad[0]
        print("  got", b1[r, cc], "dec", dec[r, cc], "b1 row", b1[r, :8].tolist())
# the test's own comparison, context as the test makes it (batch 4)
img = oracle.synth_image(0, 1080, 1920)
ref = oracle.split_planes(oracle.build_gaussian_pyramid(img), 1080, 1920, 5, 5)
for mb in (1, 4):
    c = siftgpu.Context(1080, 1920, mb, device=0, flags=1)
    for rep in range(2):
        gp = c.buildGaussianPyramid(img, 5)
        errs = [float(np.abs(p.astype(np.float64) - q).max()) for p, q in zip(gp, ref)]
        print("max_batch", mb, "rep", rep, [round(e, 5) for e in errs])
    c.close()
