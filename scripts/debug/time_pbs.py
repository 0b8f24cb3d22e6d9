"""Debug helper (GPU box): time the batched PBS stage (device-resident, 16383 bits) for the library
in TAE_LIB_PATH; results are not checked (timing variants compute garbage on purpose)."""
import os, sys, time, ctypes as C
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tfhe-aes-2_amd")]
import torch
import tfhe_aes
from tfhe_aes import _native as N
SEED = bytes(range(32))
ck, keys = tfhe_aes.generate_keys_raw(tfhe_aes.PARAMS_SQRD_LVL_64, SEED, threads=16)
ctx = tfhe_aes.context_from_raw(tfhe_aes.PARAMS_SQRD_LVL_64, keys, device=0)
B = 16383
small = torch.randint(-2**62, 2**62, (B, 678), dtype=torch.int64, device="cuda")
big = torch.empty((B, 2049), dtype=torch.int64, device="cuda")
for it in range(3):
    torch.cuda.synchronize(); ctx.synchronize()
    t = time.time()
    N.check(N.lib().tae_stage_pbs_shift_boolean(ctx._h, C.c_void_p(small.data_ptr()), B, 1, C.c_void_p(big.data_ptr()), N.TAE_MEM_DEVICE))
    ctx.synchronize()
    dt = time.time() - t
print(os.path.basename(os.environ.get("TAE_LIB_PATH", "default")), f"{dt * 1e3:.1f} ms")
