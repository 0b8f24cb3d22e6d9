"""Debug helper (GPU box): vertical packing with 0..2 input GGSWs (0 = init + sample extraction only)
for both blind-rotation kernels vs the oracle."""
import os, sys, ctypes as C
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tfhe-aes-2_amd")]
import tfhe_aes
from tfhe_aes import _native as N, aes_128
from oracle import oracle
SEED = bytes(range(32)); BIG = 2049
vp = lambda a: a.ctypes.data_as(C.c_void_p)
def stats(a, b):
    d = (a.astype(np.uint64) - b.astype(np.uint64)).view(np.int64)
    nz = np.count_nonzero(d)
    return f"{nz}/{d.size} differ, max|d| {np.abs(d).max() if nz else 0:.3e}, idx {np.flatnonzero(d)[:8]}"
oracle.build()
ok = oracle.Keys(oracle.PARAMS_SQRD_LVL_64, SEED, threads=16)
ck, keys = tfhe_aes.generate_keys_raw(tfhe_aes.PARAMS_SQRD_LVL_64, SEED, threads=16)
cts = ck.encrypt_bits_raw([1, 0, 1, 1, 0, 0, 1, 0], start_index=5000)
gf = np.concatenate([ok.ggsw_to_fourier(ok.circuit_bootstrap_boolean(ok.keyswitch(c))) for c in cts[:2]])
lut = oracle.generate_lut(512, 8, 8, lambda x: aes_128.SBOX[x])
for mode in ("512", "256"):
    os.environ["TAE_BR_256"] = "1" if mode == "256" else "0"
    ctx = tfhe_aes.context_from_raw(tfhe_aes.PARAMS_SQRD_LVL_64, keys, device=0)
    for n_in in (0, 1, 2):
        o2 = np.zeros((4, BIG), dtype=np.uint64)
        g = np.ascontiguousarray(gf[: max(n_in, 1) * len(gf) // 2]).view(np.float64)
        rc = N.lib().tae_stage_vertical_packing(ctx._h, vp(g), 1, n_in, vp(lut), 4, vp(o2), N.TAE_MEM_HOST)
        if rc:
            print(mode, n_in, "rc", rc, N.lib().tae_last_error()); continue
        for j in range(4):
            ref = ok.vertical_packing(lut[j * 512:(j + 1) * 512], gf, n_in)
            print(mode, "n_in", n_in, "out", j, stats(o2[j], ref), "got[:3]", o2[j][:3], "ref[:3]", ref[:3])
    del ctx
