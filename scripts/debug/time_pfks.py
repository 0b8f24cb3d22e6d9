"""Debug helper (GPU box): time the PFKS stage (device-resident, 16384 big LWEs -> GGSW level 1) for
the library in TAE_LIB_PATH; results are not checked."""
import os, sys, time, ctypes as C
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tfhe-aes-2_amd")]
import torch
import tfhe_aes
from tfhe_aes import _native as N
SEED = bytes(range(32))
ck, keys = tfhe_aes.generate_keys_raw(tfhe_aes.PARAMS_SQRD_LVL_64, SEED, threads=16)
ctx = tfhe_aes.context_from_raw(tfhe_aes.PARAMS_SQRD_LVL_64, keys, device=0)
B = 16384
big = torch.randint(-2**62, 2**62, (B, 2049), dtype=torch.int64, device="cuda")
ggsw = torch.empty((B, 5 * 2560), dtype=torch.int64, device="cuda")
ts = []
for it in range(5):
    torch.cuda.synchronize(); ctx.synchronize()
    t = time.time()
    N.check(N.lib().tae_stage_pfks_ggsw(ctx._h, C.c_void_p(big.data_ptr()), B, 1, C.c_void_p(ggsw.data_ptr()), N.TAE_MEM_DEVICE))
    ctx.synchronize()
    ts.append(time.time() - t)
print(os.path.basename(os.environ.get("TAE_LIB_PATH", "default")), "pfks %.2f ms" % (min(ts[1:]) * 1e3))
