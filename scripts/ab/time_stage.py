"""A/B helper (GPU box): time one blind-rotation (or PFKS) stage shape for the library in TAE_LIB_PATH
(default: the in-tree product library) and print one line `<lib> <shape> <ms> [<GHz>]`.

Shapes (inputs are random device-resident LWEs: timing variants may compute garbage on purpose, and
correct libraries are checked by the parity tests, not here):
  pbs1     1-bit model PBS stage, B = TAE_B (default 16383: br512x4 on 16128 + br512lat on 255)
  pbs1lat  1-bit model PBS stage, B = 128 (one AES block: br512lat)
  pbs8     8-bit model PBS stage, B = TAE_B (default 8192: br1024 C = 2; <= 256: br1024lat)
  pfks1    1-bit model PFKS into GGSW, B = TAE_B (default 16384)
  vp1      1-bit model vertical packing, 8 -> 24 LUT over TAE_B / 8 groups (default 2048 = 128 blocks), on the
           Fourier GGSWs of random torus GGSWs
The time is the minimum over TAE_REPS (default 3) launches after one warm-up; with TAE_CLOCK=1 one more
launch runs with the in-kernel clock stamps and its effective shader clock is printed beside it.
"""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tfhe-aes-2_amd")]
import torch  # noqa: E402  (torch's HIP runtime first, as bench.py)
import tfhe_aes  # noqa: E402
from tfhe_aes import _native as N  # noqa: E402

SEED = bytes(range(32))
shape = sys.argv[1] if len(sys.argv) > 1 else "pbs1"
pid = tfhe_aes.PARAMS_WOPPBS_8BIT if shape == "pbs8" else tfhe_aes.PARAMS_SQRD_LVL_64
default_b = {"pbs1": 16383, "pbs1lat": 128, "pbs8": 8192, "pfks1": 16384, "vp1": 16384}[shape]
B = int(os.environ.get("TAE_B", default_b))
reps = int(os.environ.get("TAE_REPS", "3"))
p = tfhe_aes.get_params(pid)
_, keys = tfhe_aes.generate_keys_raw(pid, SEED, threads=16)
ctx = tfhe_aes.context_from_raw(pid, keys, device=0)
del keys
g = torch.Generator(device="cuda").manual_seed(1)
if shape == "vp1":
    G = B // 8
    glwe = (p["k"] + 1) * p["N"]
    std = torch.randint(-2**62, 2**62, (B, p["cbs_l"] * (p["k"] + 1) * glwe), dtype=torch.int64, device="cuda", generator=g)
    gf = torch.empty((B, p["cbs_l"] * (p["k"] + 1) * (p["k"] + 1) * (p["N"] // 2) * 2), dtype=torch.float64, device="cuda")
    N.check(N.lib().tae_stage_ggsw_fourier(ctx._h, C.c_void_p(std.data_ptr()), B, C.c_void_p(gf.data_ptr()), N.TAE_MEM_DEVICE))
    del std
    lut = torch.randint(-2**62, 2**62, (24, p["N"]), dtype=torch.int64, device="cuda", generator=g)
    dst = torch.empty((G * 24, p["k"] * p["N"] + 1), dtype=torch.int64, device="cuda")
    call = lambda: N.lib().tae_stage_vertical_packing(ctx._h, C.c_void_p(gf.data_ptr()), G, 8, C.c_void_p(lut.data_ptr()),
                                                      24, C.c_void_p(dst.data_ptr()), N.TAE_MEM_DEVICE)
elif shape == "pfks1":
    src = torch.randint(-2**62, 2**62, (B, p["k"] * p["N"] + 1), dtype=torch.int64, device="cuda", generator=g)
    dst = torch.empty((B, p["cbs_l"] * (p["k"] + 1) * (p["k"] + 1) * p["N"]), dtype=torch.int64, device="cuda")
    call = lambda: N.lib().tae_stage_pfks_ggsw(ctx._h, C.c_void_p(src.data_ptr()), B, 1, C.c_void_p(dst.data_ptr()),
                                          N.TAE_MEM_DEVICE)
else:
    src = torch.randint(-2**62, 2**62, (B, p["n"] + 1), dtype=torch.int64, device="cuda", generator=g)
    dst = torch.empty((B, p["k"] * p["N"] + 1), dtype=torch.int64, device="cuda")
    call = lambda: N.lib().tae_stage_pbs_shift_boolean(ctx._h, C.c_void_p(src.data_ptr()), B, 1,
                                                       C.c_void_p(dst.data_ptr()), N.TAE_MEM_DEVICE)
ts = []
for it in range(reps + 1):
    torch.cuda.synchronize()
    ctx.synchronize()
    t = time.time()
    N.check(call())
    ctx.synchronize()
    ts.append(time.time() - t)
ghz = ""
if os.environ.get("TAE_CLOCK") == "1" and shape not in ("pfks1", "vp1"):
    ctx.set_timing(True, clock=True)
    N.check(call())
    ctx.synchronize()
    st = ctx.last_stage_times()
    ctx.set_timing(False)
    if "pbs_clock_ghz" in st:
        ghz = " %.3f GHz" % st["pbs_clock_ghz"]
lib = os.path.basename(os.environ.get("TAE_LIB_PATH", "default"))
print(f"{lib} {shape} B={B} {min(ts[1:]) * 1e3:.2f} ms{ghz}", flush=True)
