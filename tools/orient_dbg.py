import os, sys, numpy as np, torch
sys.path.insert(0, "sift-gpu_amd"); sys.path.insert(0, "oracle")
import siftgpu
R, C = 1080, 1920
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1
with siftgpu.Context(R, C, B, device=0) as ctx:
    imgs = torch.empty((B, R, C), dtype=torch.float32, device="cuda")
    ctx.synth_images(imgs.data_ptr(), B, R, C, C, R * C, seed_base=0)
    cap = B * 40000
    k = torch.empty((cap, 7), dtype=torch.int32, device="cuda"); d = torch.empty((cap, 128), dtype=torch.float32, device="cuda")
    o = torch.empty((B + 1,), dtype=torch.int32, device="cuda")
    ctx.detect_compute_batch(imgs.data_ptr(), B, R, C, C, R * C, k.data_ptr(), d.data_ptr(), cap, o.data_ptr())
    ctx.sync()
    n = int(o[1].item())
    np.save(sys.argv[1], k[:n].cpu().numpy())
