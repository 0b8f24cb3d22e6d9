#!/usr/bin/env python3
"""FHE AES-128 counter-mode throughput on MI355X (BASELINE.json metric: FHE AES-128 blocks/sec).

One step = one full 10-round homomorphic AES-128 (fhe_sbox_gal_mul_pbs::encrypt_block_for_rounds,
ShortintWoppbs1BitSboxGalMulPbsAesEncrypt, params_sqrd_lvl_64) of this rank's batch of counter blocks
(default 128 per GPU = BASELINE configs[2]; at 8 GPUs 1024 blocks = configs[3]).  Inputs (encrypted
blocks + FHE-expanded round key) are resident in HBM before the timed region; outputs are decrypted
and checked against plain AES after it.  The FHE key schedule (main.rs:130-139) runs once and is
reported separately (key_expansion_s), as in the reference.

Multi-GPU: `python -m torch.distributed.run --nproc-per-node N bench.py --gpus N`: blocks shard across
ranks (weak scaling); the server keys (KSK, BSK, PFPKSK: 672 MB) and the expanded round key are
broadcast once from rank 0 over RCCL (torch.distributed "nccl") before timing; no collective on the
data path.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "tfhe-aes-2_amd"))
sys.path.insert(0, ROOT)

SEED = bytes(range(32))
README_KEY = bytes.fromhex("76b8e0ada0f13d90405d6ae55386bd28")  # README / main.rs scenario
README_IV = bytes.fromhex("bdd219b8a08ded1a")
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md chip table (spec)
FP64_PEAK_TFLOPS = 78.6   # MI355X FP64 vector (= FP64 matrix) dense peak, spec
SPEC_CLOCK_GHZ = 2.4      # the clock the spec peaks assume
FP64_SUSTAINED_TFLOPS = 58.0  # measured sustained v_fma_f64 rate, all CUs (scripts/probes/fp64_peak.hip)
PBS_KERNELS = {"1bit": "tae::br512x4::br_kernel<3, true, 12>", "8bit": "tae::br1024w::br_kernel<6, 7>"}


def pbs_algorithmic(p, bits):
    """Per-launch algorithmic figures of the PBS kernel: the Fourier BSK streamed once,
    every small LWE read, every big LWE written; FP64 = 677 CMux x (20 FFT x (5 M log2 M + 6 M) +
    75 x M x 8) per bootstrap."""
    M = p["N"] // 2
    logM = M.bit_length() - 1
    rows = (p["k"] + 1) * p["pbs_l"]
    bsk_bytes = p["n"] * rows * (p["k"] + 1) * M * 16
    io_bytes = bits * ((p["n"] + 1) + (p["k"] * p["N"] + 1)) * 8
    ffts = rows + (p["k"] + 1)
    flop_cmux = ffts * (5 * M * logM + 6 * M) + rows * (p["k"] + 1) * M * 8
    return bsk_bytes + io_bytes, p["n"] * flop_cmux * bits


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--blocks-per-gpu", type=int, default=128)
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--key-schedule", choices=["fhe", "plain"], default="fhe")
    ap.add_argument("--cpu-baseline", choices=["auto", "on", "off"], default="auto")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads (0: this process's CPU share, capped by OMP_NUM_THREADS)")
    ap.add_argument("--single-block", choices=["auto", "on", "off"], default="auto",
                    help="also time one block alone (BASELINE configs[1]: 16 SBOX x 10 rounds on 1 GPU); "
                         "auto = on at world size 1")
    ap.add_argument("--model", choices=["1bit", "8bit"], default="1bit",
                    help="1bit: ShortintWoppbs1BitSboxGalMulPbsAesEncrypt (params_sqrd_lvl_64, the metric); "
                         "8bit: ShortintWoppbs8BitSboxPbsAesEncrypt (BASELINE config #5)")
    ap.add_argument("--model8-leg", choices=["auto", "on", "off"], default="auto",
                    help="with --model 1bit: also time BASELINE config #5 (8-bit model) on a bounded batch "
                         "(--model8-blocks blocks, one step) and report it beside the headline line; auto = on "
                         "at world size 1")
    ap.add_argument("--model8-blocks", type=int, default=64)
    ap.add_argument("--force-dist", action="store_true",
                    help="take the torch.distributed branch even at world size 1 (backend nccl = RCCL unless "
                         "TAE_BENCH_BACKEND says otherwise): communicator init, the device broadcast of the server "
                         "keys and the round key, device-built contexts, max/min over ranks; launch it under "
                         "torch.distributed.run (MASTER_ADDR / MASTER_PORT)")
    ap.add_argument("--host-buffers", choices=["auto", "on", "off"], default="auto",
                    help="one extra step with host arrays (PCIe-inclusive rate); auto = on at world 1")
    args = ap.parse_args()
    PBS_KERNEL = PBS_KERNELS[args.model]

    import torch  # plumbing: device memory + torch.distributed (nccl == RCCL)
    import tfhe_aes
    from tfhe_aes import aes_128
    from tfhe_aes import distributed as D

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU; TAE_BENCH_BACKEND=gloo rehearses the multi-rank path with several ranks on one
    # GPU (RCCL refuses two ranks on one device): same key broadcast, device-key contexts and timing
    backend = os.environ.get("TAE_BENCH_BACKEND", "nccl")
    dev = local % max(1, torch.cuda.device_count()) if backend == "gloo" else local
    torch.cuda.set_device(dev)
    dist = None
    use_dist = world > 1 or args.force_dist
    if use_dist:
        import torch.distributed as dist
        if backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
    threads = min(16, os.cpu_count() or 1)
    pid = tfhe_aes.PARAMS_SQRD_LVL_64 if args.model == "1bit" else tfhe_aes.PARAMS_WOPPBS_8BIT
    p = tfhe_aes.get_params(pid)
    L = tfhe_aes.bit_len(pid)  # one bit ciphertext: big key (1-bit model) or small key (8-bit model)
    E = (aes_128.ShortintWoppbs1BitSboxGalMulPbsAesEncrypt if args.model == "1bit"
         else aes_128.ShortintWoppbs8BitSboxPbsAesEncrypt)

    # ---- keys: generated on rank 0 (client side), server keys broadcast once over RCCL ----
    t = time.time()
    sizes = None
    if rank == 0:
        ck0, raw = tfhe_aes.generate_keys_raw(pid, SEED, threads=threads)
    keygen_s = time.time() - t
    ck = tfhe_aes.client_key_from_seed(pid, SEED)
    t = time.time()
    dist_info = None
    if not dist:
        ctx = tfhe_aes.context_from_raw(pid, raw, device=dev)
    else:
        from tfhe_aes import _native as N
        lens = [C.c_size_t() for _ in range(3)]
        N.check(N.lib().tae_server_key_sizes(pid, *[C.byref(x) for x in lens]))
        bufs = D.broadcast_u64(dist, raw if rank == 0 else None, [x.value for x in lens], rank, f"cuda:{dev}")
        torch.cuda.synchronize()
        bcast_s = time.time() - t
        ctx = tfhe_aes.context_from_raw(pid, [b.data_ptr() for b in bufs], device=dev, mem=1)
        ctx._keepalive = bufs
        dist_info = {"backend": dist.get_backend(), "world": world, "server_key_bytes": int(sum(b.numel() * 8 for b in bufs)),
                     "server_key_broadcast_s": bcast_s, "key_tensors_on": str(bufs[0].device)}
    key_setup_s = time.time() - t

    # ---- expanded key: FHE key schedule on rank 0 (timed separately), broadcast ----
    t = time.time()
    rk_np = None
    if rank == 0:
        if args.key_schedule == "fhe":
            key_bits = aes_128.encrypt_byte_array(ck, README_KEY)
            ek = E.key_schedule(ctx, key_bits)
            rk_np = np.stack([b.data(L) for w in ek for byte in w for b in byte])
            assert b"".join(aes_128.decrypt_byte_array(ck, w) for w in ek) == b"".join(
                aes_128.key_schedule_plain(README_KEY)), "FHE key schedule mismatch"
        else:
            ek = b"".join(aes_128.key_schedule_plain(README_KEY))
            rk_np = ck.encrypt_bits_raw([b for byte in ek for b in aes_128.u8_to_bits(byte)])  # fresh indices
    key_expansion_s = time.time() - t
    if rank == 0:
        rk_dev = torch.from_numpy(rk_np.view(np.int64)).to(f"cuda:{dev}")
    else:
        rk_dev = torch.empty((44 * 32, L), dtype=torch.int64, device=f"cuda:{dev}")
    if dist:
        dist.broadcast(rk_dev, src=0)

    # ---- this rank's counter blocks (main.rs:108-115), encrypted client side, resident in HBM ----
    nb = args.blocks_per_gpu
    blocks = D.counter_blocks_for_rank(README_IV, rank, world, nb)
    t = time.time()
    bits = aes_128.blocks_to_bits(blocks)
    cts = ck.encrypt_bits_raw(bits, start_index=D.encrypt_start_index(rank, nb))
    encrypt_s = time.time() - t
    blk_dev = torch.from_numpy(cts.view(np.int64)).to(f"cuda:{dev}")
    out_dev = torch.empty_like(blk_dev)
    torch.cuda.synchronize()

    def step(o=out_dev):
        E.encrypt_blocks_device(ctx, rk_dev.data_ptr(), blk_dev.data_ptr(), nb, args.rounds, o.data_ptr())

    for _ in range(args.warmup):
        step()
    ctx.set_timing(True)
    stage_ms = {}
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    ctx.synchronize()
    t0 = time.time()
    for _ in range(args.steps):
        step()
        for kk, v in ctx.last_stage_times().items():
            stage_ms[kk] = stage_ms.get(kk, 0.0) + v
    ctx.synchronize()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.time() - t0
    ctx.set_timing(False)
    if dist:
        elapsed = D.max_over_ranks(dist, elapsed, f"cuda:{dev}")
    # the timed steps' own output, copied out before anything else writes a ciphertext buffer
    out = out_dev.cpu().numpy().view(np.uint64)
    # effective shader clock of the PBS launches: one more step, right after the timed ones (chip warm),
    # with in-kernel clock stamps (a diagnostic mode: each stamped launch is read back synchronously), into
    # its own output buffer; its ciphertexts must equal the timed steps' bit for bit
    clk_out = torch.empty_like(out_dev)
    ctx.set_timing(True, clock=True)
    step(clk_out)
    ctx.synchronize()
    clk = ctx.last_stage_times()
    ctx.set_timing(False)
    clock_ghz = clk.get("pbs_clock_ghz")
    clock_step_identical = bool(np.array_equal(clk_out.cpu().numpy().view(np.uint64), out))
    del clk_out

    # ---- correctness gate on the timed steps' output: decrypt and compare with plain AES ----
    got = aes_128.bits_to_blocks(ck.decrypt_bits_raw(out))
    ek_plain = aes_128.key_schedule_plain(README_KEY)
    ok = int(all(g == aes_128.encrypt_block_plain(ek_plain, b, args.rounds) for g, b in zip(got, blocks)))
    if not clock_step_identical:  # the stamped step must reproduce the timed steps' ciphertexts bit for bit
        print(f"rank {rank}: the clock-stamped step's ciphertexts differ from the timed steps'", file=sys.stderr)
        ok = 0
    if dist:
        ok = D.min_over_ranks(dist, ok, f"cuda:{dev}")
    if not ok:
        raise SystemExit(f"rank {rank}: decrypted AES output differs from plain AES")

    # ---- BASELINE configs[1]: one block alone (latency; not the headline value) ----
    single = None
    if args.single_block == "on" or (args.single_block == "auto" and world == 1):
        one_dev = blk_dev[:128].contiguous()
        one_out = torch.empty_like(one_dev)

        def one():
            E.encrypt_blocks_device(ctx, rk_dev.data_ptr(), one_dev.data_ptr(), 1, args.rounds, one_out.data_ptr())
        one()
        ctx.synchronize()
        reps, t1 = 3, time.time()
        for _ in range(reps):
            one()
        ctx.synchronize()
        lat = (time.time() - t1) / reps
        ctx.set_timing(True)  # one more call, outside the timed reps: where the latency goes
        one()
        ctx.synchronize()
        one_stages = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in ctx.last_stage_times().items()}
        ctx.set_timing(False)
        got1 =aes_128.bits_to_blocks(ck.decrypt_bits_raw(one_out.cpu().numpy().view(np.uint64)))[0]
        single = {"config": "1 block, 16 SBOX x %d rounds on 1 GPU" % args.rounds, "s_per_block": lat,
                  "blocks_per_s": 1.0 / lat, "per_sbox_ms": lat * 1e3 / (16 * args.rounds),
                  "stage_ms": one_stages,
                  "correct": got1 == aes_128.encrypt_block_plain(aes_128.key_schedule_plain(README_KEY), blocks[0],
                                                                 args.rounds)}

    # ---- host buffers: one step through tae_aes_encrypt_blocks_raw with host arrays (PCIe copies of
    # the expanded key, blocks and results included); reported beside `value`, never as it ----
    host_io = None
    if args.host_buffers == "on" or (args.host_buffers == "auto" and world == 1):
        blocks_h = cts.reshape(nb, 128, L)
        t1 = time.time()
        out_h = E.encrypt_blocks_raw(ctx, rk_np, blocks_h, args.rounds)
        dt = time.time() - t1
        host_io = {"config": f"{nb} blocks x {args.rounds} rounds, host arrays in and out (one step)",
                   "s_per_step": dt, "blocks_per_s": nb / dt,
                   "copy_bytes": int(rk_np.nbytes + blocks_h.nbytes + out_h.nbytes),
                   "identical_to_device_path": bool(np.array_equal(out_h.reshape(out.shape), out))}

    total_blocks = nb * world * args.steps
    value = total_blocks / elapsed
    ms_per_step = elapsed * 1000.0 / args.steps

    # ---- roofline of the dominant kernel (PBS = homomorphic_shift_boolean blind rotation) ----
    # Its own launches (ctx timing "pbs_main": the throughput kernel alone, HIP events on the engine
    # stream around each launch) give the roofline; the whole PBS stage (plus the small-batch
    # remainder kernel) is reported beside it.
    launches = stage_ms.get("pbs_launches", 0)
    pbs_ms = stage_ms.get("pbs", 0.0) / max(launches, 1)
    main_ms = stage_ms.get("pbs_main", 0.0) / max(launches, 1)
    main_cts = stage_ms.get("pbs_main_cts", 0.0) / max(launches, 1)
    bytes_launch, flop_launch = pbs_algorithmic(p, nb * 16 * 8)
    if main_ms > 0 and main_cts > 0:  # 1-bit model: br512x4 launches
        k_bytes, k_flop = pbs_algorithmic(p, int(main_cts))
        k_ms = main_ms
    else:  # one kernel covers the whole stage
        k_bytes, k_flop, k_ms = bytes_launch, flop_launch, pbs_ms
    gbs = k_bytes / (k_ms * 1e-3) / 1e9 if k_ms > 0 else None
    tflops = k_flop / (k_ms * 1e-3) / 1e12 if k_ms > 0 else None
    stage_tflops = flop_launch / (pbs_ms * 1e-3) / 1e12 if pbs_ms > 0 else None
    # HBM traffic per launch of the same kernel from the committed PMC pass (scripts/bench_profile.sh
    # -> scripts/prof_summary.py: 2 x FETCH_SIZE + WRITE_SIZE), valid only for the same batch shape.
    traffic, traffic_src = None, None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_latest.json")
    if args.model == "1bit" and os.path.exists(pmc_path):
        with open(pmc_path) as fh:
            pm = json.load(fh)
        ent = pm.get("kernels", {}).get(PBS_KERNEL, {})
        if pm.get("blocks_per_gpu") == nb and "hbm_bytes_per_launch" in ent:
            traffic, traffic_src = ent["hbm_bytes_per_launch"], pm.get("source")
    pmc8_path = os.path.join(ROOT, "profiles", "pmc8_latest.json")
    if args.model == "8bit" and os.path.exists(pmc8_path):
        # scripts/prof8.sh -> scripts/prof_split_summary.py, split per launch shape: the CBS launch is the
        # kernel's largest grid
        with open(pmc8_path) as fh:
            pm = json.load(fh)
        ents = [e for e in pm.get("launches", {}).values() if e.get("kernel") == PBS_KERNEL]
        ent = max(ents, key=lambda e: e["grid_threads"]) if ents else {}
        if pm.get("blocks_per_gpu") == nb and "traffic_bytes_per_launch" in ent:
            traffic, traffic_src = ent["traffic_bytes_per_launch"], pm.get("source")
    # The batched blind rotation is bound by the FP64 vector ALU (>= 10 flop/B at any
    # batch; no MFMA on this path): peak = the dense FP64 vector rate, HBM figures ride along.
    roofline = {"bound": "fp64_valu", "achieved": tflops, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": (tflops / FP64_PEAK_TFLOPS) if tflops else None, "traffic": traffic,
                "traffic_unit": "bytes/launch", "traffic_source": traffic_src,
                "traffic_note": "L2-miss bytes (2 x FETCH_SIZE + WRITE_SIZE, MI355X_MICROARCH.md): they include "
                                "Infinity-Cache hits, and no counter here separates the bytes that reached HBM",
                "kernel": PBS_KERNEL + " (homomorphic_shift_boolean blind rotation)", "avg_launch_ms": k_ms,
                "ciphertexts_per_launch": main_cts if main_ms > 0 else nb * 16 * 8,
                "algorithmic_flop_per_launch": k_flop,
                "stage": {"avg_ms": pbs_ms, "ciphertexts": nb * 16 * 8, "achieved": stage_tflops,
                          "frac": (stage_tflops / FP64_PEAK_TFLOPS) if stage_tflops else None,
                          "note": ("whole PBS stage per launch: the kernel above + the br512lat remainder" if main_ms > 0
                                   else "whole PBS stage per launch: the kernel above alone")},
                "hbm": {"achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": (gbs / HBM_PEAK_GBS) if gbs else None,
                        "algorithmic_bytes_per_launch": k_bytes},
                "sustained": {"peak": FP64_SUSTAINED_TFLOPS, "frac": (tflops / FP64_SUSTAINED_TFLOPS) if tflops else None,
                              "note": "v_fma_f64 rate the chip holds with every CU busy "
                                      "(scripts/probes/fp64_peak.hip); the spec peak assumes 2.4 GHz"},
                "effective_clock_ghz": clock_ghz, "clock_step_identical": clock_step_identical,
                "at_clock": at_clock(tflops, clock_ghz)}
    stage_share = {k: v / args.steps for k, v in stage_ms.items() if k not in ("pbs_launches", "pbs_main_cts")}

    cpu = None
    want_cpu = args.cpu_baseline == "on" or (args.cpu_baseline == "auto" and world == 1)
    if want_cpu and rank == 0:
        cpu = cpu_baseline(raw, ck, args.cpu_threads or cpu_share(), args.model, rk_np)

    model8 = None
    want8 = args.model == "1bit" and (args.model8_leg == "on" or (args.model8_leg == "auto" and world == 1))
    if want8 and rank == 0:
        model8 = model8_leg(torch, dev, args.model8_blocks, threads)

    if rank == 0:
        rec = {"metric": "FHE AES-128 blocks/sec", "value": value, "unit": "blocks/s", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
               "config": {"workload": f"{nb} counter-mode blocks per GPU, {args.rounds}-round FHE AES-128 ("
                                      + ("ShortintWoppbs1BitSboxGalMulPbsAesEncrypt, params_sqrd_lvl_64)"
                                         if args.model == "1bit" else
                                         "ShortintWoppbs8BitSboxPbsAesEncrypt, shortint_woppbs_8bit params)"),
                          "model": args.model,
                          "blocks_per_gpu": nb, "global_blocks": nb * world, "rounds": args.rounds,
                          "parallelism": f"blocks sharded over {world} GPU(s), keys broadcast once"},
               "roofline": roofline, "cpu_baseline": cpu,
               "stage_ms_per_step": stage_share, "per_sbox_ms": ms_per_step / (nb * 16 * args.rounds),
               "keygen_s": keygen_s, "key_setup_s": key_setup_s, "key_expansion_s": key_expansion_s,
               "encrypt_s": encrypt_s, "correct": bool(ok), "single_block": single, "host_buffers": host_io,
               "model8": model8, "dist": dist_info}
        print(json.dumps(rec), flush=True)
    if dist:
        dist.destroy_process_group()


def at_clock(tflops, ghz):
    """The FP64 spec peak scaled to the clock the launches actually ran at (the spec assumes 2.4 GHz):
    what the kernel's cycles reach at that clock, separable from the chip's DVFS give-back."""
    if not tflops or not ghz:
        return None
    peak = FP64_PEAK_TFLOPS * ghz / SPEC_CLOCK_GHZ
    return {"peak": peak, "frac": tflops / peak,
            "note": "in-kernel s_memtime / s_memrealtime stamps of the PBS launches of one extra step after the "
                    "timed ones (median over workgroups, mean over launches; MI355X_MICROARCH.md DVFS give-back)"}


def cpu_share():
    """Threads for the CPU baseline: this process's CPU share (affinity mask), capped by
    OMP_NUM_THREADS where the job scheduler sets it (the GPU box gives a 1-GPU job 16 host threads
    while os.cpu_count() reports the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    cap = os.environ.get("OMP_NUM_THREADS")
    if cap and cap.isdigit() and int(cap) > 0:
        n = min(n, int(cap))
    return max(1, n)


def cpu_baseline(raw, ck, threads, model="1bit", rk=None):
    """CPU oracle (restatement, kind "port": tfhe-rs is absent here) timed on this process's host cores:
    one full 10-round block (fhe_sbox_gal_mul_pbs::encrypt_block_for_rounds) measured directly, the 16
    SBOX circuit bootstraps of each round run on `threads` threads as the reference's rayon splits a
    block's bytes (fhe_sbox_gal_mul_pbs.rs:33-41; the 8 extract-bit keyswitches of each SBOX are a
    negligible share).  At N = 128 the reference's rayon over blocks (main.rs:148-152) keeps the same
    cores busy, so its throughput is extrapolated from the per-block time at the same core count."""
    from oracle import oracle
    from tfhe_aes import aes_128
    ok = oracle.Keys(oracle.PARAMS_SQRD_LVL_64 if model == "1bit" else oracle.PARAMS_WOPPBS_8BIT, None, raw=raw)
    blk = README_IV + (1).to_bytes(8, "big")
    cts = ck.encrypt_bits_raw(aes_128.blocks_to_bits([blk]))  # fresh indices
    if rk is None:
        ek = b"".join(aes_128.key_schedule_plain(README_KEY))
        rk = ck.encrypt_bits_raw([b for byte in ek for b in aes_128.u8_to_bits(byte)])
    rounds = 10
    t = time.time()
    if model == "1bit":
        out = ok.aes_encrypt_block(rk, cts, rounds, threads=threads)
    else:
        out = ok.aes8_encrypt_block(rk, cts, rounds, threads=threads)
    dt = time.time() - t
    correct = aes_128.bits_to_blocks(ck.decrypt_bits_raw(out))[0] == aes_128.encrypt_block_plain(
        aes_128.key_schedule_plain(README_KEY), blk, rounds)
    return {"value": 1.0 / dt, "unit": "blocks/s", "cores": threads, "kind": "port",
            "nproc": os.cpu_count(), "cpu_share": cpu_share(), "correct": bool(correct),
            "extrapolated_128_blocks_per_s": 1.0 / dt,
            "sample": f"1 block x {rounds} rounds measured directly ({dt:.2f} s; 16 SBOX "
                      + ("8->24 circuit bootstraps" if model == "1bit" else "bootstrap_with_lut") +
                      f" per round on {threads} threads, oracle/tfhe_oracle.c); the 128-block figure is "
                      "extrapolated (blocks independent, same cores)"}


def model8_leg(torch, dev, nb, threads, steps=3):
    """BASELINE configs[4] (ShortintWoppbs8BitSboxPbsAesEncrypt, shortint_woppbs_8bit params) on a bounded
    batch: nb counter blocks, one warm-up and `steps` timed 10-round steps (mean, with their spread),
    decrypted against plain AES."""
    import tfhe_aes
    from tfhe_aes import aes_128
    from tfhe_aes import distributed as D
    pid = tfhe_aes.PARAMS_WOPPBS_8BIT
    t = time.time()
    ck, raw = tfhe_aes.generate_keys_raw(pid, SEED, threads=threads)
    ctx = tfhe_aes.context_from_raw(pid, raw, device=dev)
    del raw
    setup_s = time.time() - t
    L = tfhe_aes.bit_len(pid)
    E8 = aes_128.ShortintWoppbs8BitSboxPbsAesEncrypt
    ek = b"".join(aes_128.key_schedule_plain(README_KEY))
    rk = ck.encrypt_bits_raw([b for byte in ek for b in aes_128.u8_to_bits(byte)])
    blocks = D.counter_blocks_for_rank(README_IV, 0, 1, nb)
    cts = ck.encrypt_bits_raw(aes_128.blocks_to_bits(blocks))
    rk_dev = torch.from_numpy(rk.view(np.int64)).to(f"cuda:{dev}")
    blk_dev = torch.from_numpy(cts.view(np.int64)).to(f"cuda:{dev}")
    out_dev = torch.empty_like(blk_dev)
    torch.cuda.synchronize()
    step = lambda o: E8.encrypt_blocks_device(ctx, rk_dev.data_ptr(), blk_dev.data_ptr(), nb, 10, o.data_ptr())
    step(out_dev)
    ctx.synchronize()
    times, acc = [], {}
    ctx.set_timing(True)  # HIP events around each stage on the engine stream (no host round trips)
    for _ in range(steps):
        t0 = time.time()
        step(out_dev)
        ctx.synchronize()
        times.append(time.time() - t0)
        for kk, v in ctx.last_stage_times().items():
            acc[kk] = acc.get(kk, 0) + v
    ctx.set_timing(False)
    dt = sum(times) / len(times)
    out = out_dev.cpu().numpy().view(np.uint64)  # the timed steps' output, gated below
    # one more step with in-kernel clock stamps into its own buffer: the effective clock only
    clk_out = torch.empty_like(out_dev)
    ctx.set_timing(True, clock=True)
    step(clk_out)
    ctx.synchronize()
    clock_ghz = ctx.last_stage_times().get("pbs_clock_ghz")
    ctx.set_timing(False)
    clock_step_identical = bool(np.array_equal(clk_out.cpu().numpy().view(np.uint64), out))
    stages = {k: (round(v / steps, 1) if isinstance(v, float) else v // steps) for k, v in acc.items()
              if k not in ("pbs_main", "pbs_main_cts", "pbs_clock_ghz", "pbs_clock_launches")}
    got = aes_128.bits_to_blocks(ck.decrypt_bits_raw(out))
    ek_plain = aes_128.key_schedule_plain(README_KEY)
    correct = all(g == aes_128.encrypt_block_plain(ek_plain, b, 10) for g, b in zip(got, blocks))
    if not clock_step_identical:
        print("model8: the clock-stamped step's ciphertexts differ from the timed steps'", file=sys.stderr)
        correct = False
    del ctx, clk_out
    # the circuit bootstrap's PBS launches (one per CBS level and round, nb x 16 x 8 bits each): the
    # dominant kernel of this model, against the same FP64 spec as the headline line
    _, flop_launch = pbs_algorithmic(tfhe_aes.get_params(pid), nb * 16 * 8)
    pbs_ms, launches = stages.get("pbs", 0.0), stages.get("pbs_launches", 0)
    tf = launches * flop_launch / (pbs_ms * 1e-3) / 1e12 if pbs_ms and launches else None
    cbs_roofline = {"bound": "fp64_valu", "kernel": PBS_KERNELS["8bit"] + " (CBS PBS)",
                    "achieved": tf, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                    "frac": (tf / FP64_PEAK_TFLOPS) if tf else None, "launches_per_step": launches,
                    "algorithmic_flop_per_launch": flop_launch,
                    "avg_launch_ms": pbs_ms / launches if launches else None,
                    "effective_clock_ghz": clock_ghz, "at_clock": at_clock(tf, clock_ghz),
                    "clock_step_identical": clock_step_identical,
                    "note": "stage time per timed step over its PBS launches (HIP events on the engine stream); the "
                            "clock comes from one extra stamped step"}
    return {"config": f"ShortintWoppbs8BitSboxPbsAesEncrypt, {nb} counter blocks x 10 rounds on 1 GPU "
                      f"(BASELINE configs[4]); 1 warm-up + {steps} timed steps", "blocks": nb, "s_per_step": dt,
            "s_per_step_each": times, "spread": (max(times) - min(times)) / dt,
            "value": nb / dt, "unit": "blocks/s", "bit_len": L, "setup_s": setup_s, "stage_ms": stages,
            "cbs_pbs_roofline": cbs_roofline, "correct": bool(correct)}


if __name__ == "__main__":
    main()
