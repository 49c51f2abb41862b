"""Where does mmpde_resample_bilinear differ from the fp32 restatement?"""
import sys
import numpy as np
import torch
sys.path[:0] = ["/root/repo", "/root/repo/mm-pde_amd"]
from mmpde_amd import ops  # noqa: E402
import importlib.util  # noqa: E402
spec = importlib.util.spec_from_file_location("t", "/root/repo/tests/test_gpu_dmm_api.py")
m = importlib.util.module_from_spec(spec)
spec.loader.exec_module(m)
g = torch.Generator().manual_seed(32)
u = torch.randn(3, 48, 48, generator=g)
got = ops.resample_bilinear(u.cuda(), 32, 40).cpu()
ref = m._bilinear_f32(u, 32, 40)
d = (got - ref).abs()
idx = np.unravel_index(int(d.argmax()), d.shape)
print("max", float(d.max()), "at", idx, "rows with err>1e-6:", sorted(set(np.nonzero(d.numpy() > 1e-6)[1].tolist())),
      "cols:", sorted(set(np.nonzero(d.numpy() > 1e-6)[2].tolist())))
# constant-along-x input: isolates the y coordinate
uy = torch.arange(48, dtype=torch.float32)[:, None].repeat(1, 48)[None]
gy = ops.resample_bilinear(uy.cuda(), 32, 40).cpu()[0, :, 0]
print("y coords gpu:", gy.tolist())
ux = torch.arange(48, dtype=torch.float32)[None, :].repeat(48, 1)[None]
gx = ops.resample_bilinear(ux.cuda(), 32, 40).cpu()[0, 0, :]
print("x coords gpu:", gx.tolist())
pl, oy, ox = (int(v) for v in idx)
f = np.float32
sy, sx = f(47) / f(31), f(47) / f(39)
fy, fx = f(sy * f(oy)), f(sx * f(ox))
y0, x0 = int(fy), int(fx)
y1, x1 = min(y0 + 1, 47), min(x0 + 1, 47)
x = u.numpy()[pl]
print("fy fx", float(fy), float(fx), "y0 x0", y0, x0, "abcd", x[y0, x0], x[y0, x1], x[y1, x0], x[y1, x1])
print("gpu", float(got[pl, oy, ox]), "ref", float(ref[pl, oy, ox]))
# the same element computed from single-element planes on the GPU
one = torch.zeros(1, 48, 48)
one[0, y0, x0] = 1.0
print("weight a (gpu)", float(ops.resample_bilinear(one.cuda(), 32, 40).cpu()[0, oy, ox]),
      "f32", float((f(1) - (fy - f(y0))) * (f(1) - (fx - f(x0)))))
