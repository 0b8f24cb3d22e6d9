"""A/B helper (GPU box): one round of Shortint1BitSboxPbsAesEncrypt (fhe_impls/shortint_1bit.rs:52-72) over
nb blocks (TAE_NB, default 64), i.e. 16 nb S-box selector trees of 8 functions x 8 bits; prints the time of the
round (min over TAE_REPS after a warm-up) for the selector-tree chunk size in effect (TAE_S1_ROWS)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tfhe-aes-2_amd")]
import torch  # noqa: E402,F401  (torch's HIP runtime first, as bench.py)
import tfhe_aes  # noqa: E402
from tfhe_aes import aes_128  # noqa: E402

nb = int(os.environ.get("TAE_NB", "8"))
reps = int(os.environ.get("TAE_REPS", "1"))
ck, keys = tfhe_aes.generate_keys_raw(tfhe_aes.PARAMS_SHORTINT_1BIT, bytes(range(32)), threads=16)
ctx = tfhe_aes.context_from_raw(tfhe_aes.PARAMS_SHORTINT_1BIT, keys, device=0)
E = aes_128.Shortint1BitSboxPbsAesEncrypt
key, iv = bytes.fromhex("76b8e0ada0f13d90405d6ae55386bd28"), bytes.fromhex("bdd219b8a08ded1a")
blocks = aes_128.counter_blocks(iv, nb)
ek = b"".join(aes_128.key_schedule_plain(key))
rk = ck.encrypt_bits_raw([b for byte in ek for b in aes_128.u8_to_bits(byte)], start_index=10_000)
cts = ck.encrypt_bits_raw(aes_128.blocks_to_bits(blocks), start_index=20_000).reshape(nb, 128, -1)
ts = []
print("keys ready", flush=True)
for _ in range(reps + 1):
    t = time.time()
    out = E.encrypt_blocks_raw(ctx, rk, cts, rounds=1)
    ts.append(time.time() - t)
    print(f"  round {ts[-1]:.2f} s", flush=True)
ok = aes_128.bits_to_blocks(ck.decrypt_bits_raw(out)) == aes_128.expand_key_and_encrypt_blocks(key, blocks, 1)
print(f"s1 round nb={nb} rows={os.environ.get('TAE_S1_ROWS', 'default')} {min(ts[1:]) * 1e3:.1f} ms correct={ok}", flush=True)
