"""Debug helper (GPU box): time the 8-bit model's PBS stage (N = 1024, pbs 6 x 2^7) on TAE_PBS_B small-key
LWEs for the library in TAE_LIB_PATH; results are not checked."""
import os, sys, time, ctypes as C
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tfhe-aes-2_amd")]
import torch
import tfhe_aes
from tfhe_aes import _native as N
SEED = bytes(range(32))
B = int(os.environ.get("TAE_PBS_B", "8192"))
pid = tfhe_aes.PARAMS_WOPPBS_8BIT
ck, keys = tfhe_aes.generate_keys_raw(pid, SEED, threads=16)
ctx = tfhe_aes.context_from_raw(pid, keys, device=0)
p = tfhe_aes.get_params(pid)
small = torch.randint(-2**62, 2**62, (B, p["n"] + 1), dtype=torch.int64, device="cuda")
big = torch.empty((B, p["k"] * p["N"] + 1), dtype=torch.int64, device="cuda")
ts = []
for it in range(3):
    torch.cuda.synchronize(); ctx.synchronize()
    t = time.time()
    N.check(N.lib().tae_stage_pbs_shift_boolean(ctx._h, C.c_void_p(small.data_ptr()), B, 1, C.c_void_p(big.data_ptr()), N.TAE_MEM_DEVICE))
    ctx.synchronize()
    ts.append(time.time() - t)
print(os.path.basename(os.environ.get("TAE_LIB_PATH", "default")), f"B={B}", "pbs8 %.2f ms" % (min(ts[1:]) * 1e3))
