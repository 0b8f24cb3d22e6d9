"""Probe (verdict r05 item 4): price running the non-PBS stages of a circuit bootstrap beside the PBS on disjoint CU
sets (hipExtStreamCreateWithCUMask, the engine's TAE_CU_MASK knob), before building a chunked pipeline.

The two kernels cannot share a CU (br512x4 uses 143.5 KB of LDS, the PFKS GEMM ring 160 KiB), so an overlapped
pipeline runs chunk i+1's PBS on P CUs while chunk i's PFKS (the largest of the other stages: 130 of the 183 ms
per step) runs on the remaining 256 - P.  Timing-only: random device-resident inputs (time_stage.py's), one
16384-bootstrap stage each (one CBS launch of the 128-block bench step).  Prints, per split, the PBS stage on P
CUs, the PFKS on 256 - P CUs, both concurrently (two contexts, two host threads), against the serial sum on all
CUs.  usage (GPU box): python scripts/probes/stage_overlap.py [P ...]"""
import ctypes as C
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tfhe-aes-2_amd")]
import torch  # noqa: E402  (torch's HIP runtime first, as bench.py)
import tfhe_aes  # noqa: E402
from tfhe_aes import _native as N  # noqa: E402

B = int(os.environ.get("TAE_B", "16384"))
REPS = int(os.environ.get("TAE_REPS", "3"))
pid = tfhe_aes.PARAMS_SQRD_LVL_64
p = tfhe_aes.get_params(pid)
_, keys = tfhe_aes.generate_keys_raw(pid, bytes(range(32)), threads=16)
g = torch.Generator(device="cuda").manual_seed(1)
small = torch.randint(-2**62, 2**62, (B, p["n"] + 1), dtype=torch.int64, device="cuda", generator=g)
big = torch.randint(-2**62, 2**62, (B, p["k"] * p["N"] + 1), dtype=torch.int64, device="cuda", generator=g)
pbs_out = torch.empty((B, p["k"] * p["N"] + 1), dtype=torch.int64, device="cuda")
ggsw = torch.empty((B, p["cbs_l"] * (p["k"] + 1) * (p["k"] + 1) * p["N"]), dtype=torch.int64, device="cuda")
torch.cuda.synchronize()


def context(mask):
    if mask:
        os.environ["TAE_CU_MASK"] = mask
    else:
        os.environ.pop("TAE_CU_MASK", None)
    try:
        ctx = tfhe_aes.context_from_raw(pid, keys, device=0)
    finally:
        os.environ.pop("TAE_CU_MASK", None)
    # a caller stream of its own: the device-memory stage entry points then order after an event on that
    # stream instead of hipDeviceSynchronize (which would serialise the two contexts' launches)
    ctx.set_caller_stream(torch.cuda.Stream())
    return ctx


def pbs(ctx):
    N.check(N.lib().tae_stage_pbs_shift_boolean(ctx._h, C.c_void_p(small.data_ptr()), B, 1,
                                                C.c_void_p(pbs_out.data_ptr()), N.TAE_MEM_DEVICE))


def pfks(ctx):
    N.check(N.lib().tae_stage_pfks_ggsw(ctx._h, C.c_void_p(big.data_ptr()), B, 1, C.c_void_p(ggsw.data_ptr()),
                                        N.TAE_MEM_DEVICE))


def best(fn):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(REPS):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    return min(ts)


def both(ca, cb):
    def run():
        ta = threading.Thread(target=pbs, args=(ca,))
        tb = threading.Thread(target=pfks, args=(cb,))
        ta.start()
        tb.start()
        ta.join()
        tb.join()
    return run


full = context(None)
t_pbs, t_pf = best(lambda: pbs(full)), best(lambda: pfks(full))
print(f"all 256 CUs: PBS {t_pbs:.2f} ms, PFKS {t_pf:.2f} ms, serial {t_pbs + t_pf:.2f} ms (B = {B})", flush=True)
del full
for P in [int(a) for a in sys.argv[1:]] or [224, 208]:
    ca, cb = context(f"lo:{P}"), context(f"hi:{256 - P}")
    a, b = best(lambda: pbs(ca)), best(lambda: pfks(cb))
    ab = best(both(ca, cb))
    print(f"split {P}/{256 - P}: PBS alone {a:.2f} ms, PFKS alone {b:.2f} ms, concurrent {ab:.2f} ms "
          f"({(ab / (t_pbs + t_pf) - 1) * 100:+.1f}% vs serial on all CUs)", flush=True)
    del ca, cb
