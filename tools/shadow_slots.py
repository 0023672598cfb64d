"""Lane utilisation at shadow-query entry (debug build with RT_DBG_SHADOW_SLOTS,
loaded via RTGPU_LIB): shadow queries / (64 x waves that issued one)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "raytracing-gpu_amd"))
import rtgpu
s = rtgpu.Scene.synthetic(32, 32, 9766, seed=0x5EED, width=3840, height=2160)
ctx = rtgpu.Context(s, "octree_gpu")
import numpy as np
img, st = ctx.render_image(s.frame())
print({k: st[k] for k in ("closest", "shadow", "hits", "zero_normal")},
      "entry lane utilisation", st["shadow"] / max(1, st["zero_normal"]))
