"""Debug helper (GPU box): with lib_dump.so, both blind-rotation kernels return their LDS spectrum
buffer after step 0 / first level pass B instead of a result; compare them."""
import os, sys, ctypes as C
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tfhe-aes-2_amd")]
DUMP = int(sys.argv[1][0])
MODE = sys.argv[2] if len(sys.argv) > 2 else "pbs"
os.environ["TAE_LIB_PATH"] = os.path.join(ROOT, "tfhe-aes-2_amd", "dbg", f"lib_dump{sys.argv[1]}.so")
import tfhe_aes
from tfhe_aes import _native as N
from oracle import oracle
SEED = bytes(range(32)); BIG = 2049
vp = lambda a: a.ctypes.data_as(C.c_void_p)
oracle.build()
ok = oracle.Keys(oracle.PARAMS_SQRD_LVL_64, SEED, threads=16)
ck, keys = tfhe_aes.generate_keys_raw(tfhe_aes.PARAMS_SQRD_LVL_64, SEED, threads=16)
cts = ck.encrypt_bits_raw([1, 0, 1, 1, 0, 0, 1, 0], start_index=5000)
small = np.stack([ok.keyswitch(cts[i]) for i in range(4)])
res = {}
for mode in ("512", "256"):
    os.environ["TAE_BR_256"] = "1" if mode == "256" else "0"
    ctx = tfhe_aes.context_from_raw(tfhe_aes.PARAMS_SQRD_LVL_64, keys, device=0)
    out = np.zeros((4, BIG), dtype=np.uint64)
    if MODE == "pbs":
        N.check(N.lib().tae_stage_pbs_shift_boolean(ctx._h, vp(small), 4, 1, vp(out), N.TAE_MEM_HOST))
    else:
        from tfhe_aes import aes_128
        gf = np.concatenate([ok.ggsw_to_fourier(ok.circuit_bootstrap_boolean(ok.keyswitch(c))) for c in cts[:1]])
        lut = oracle.generate_lut(512, 8, 8, lambda x: aes_128.SBOX[x])
        g = np.ascontiguousarray(gf).view(np.float64)
        N.check(N.lib().tae_stage_vertical_packing(ctx._h, vp(g), 1, 1, vp(lut), 4, vp(out), N.TAE_MEM_HOST))
    res[mode] = out.reshape(-1)[: 15 * 272 * 2].view(np.float64).reshape(15, 272, 2) if DUMP != 4 else out.reshape(-1)[: 15 * 528]
    del ctx
a, b = res["512"], res["256"]
if DUMP == 4:
    for job in range(15):
        d = np.flatnonzero(a[job * 528: job * 528 + 512] != b[job * 528: job * 528 + 512])
        print("acc", job, "differ at", len(d), d[:12])
    sys.exit(0)
for job in range(15):
    pos = [q + (q >> 4) for q in range(256)]
    aa, bb = a[job, pos], b[job, pos]
    diff = np.flatnonzero(np.any(aa != bb, axis=1))
    print(job, "differ at", len(diff), "positions", diff.tolist() if job == 4 else diff[:10], "| new", aa[diff[:2]].tolist() if len(diff) else "", "old", bb[diff[:2]].tolist() if len(diff) else "")
