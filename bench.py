#!/usr/bin/env python3
"""PBS/s benchmark — BASELINE.json metric: "PBS/sec at TFHE 128-bit default (N=1024), batch=4096".

One step = one full programmable bootstrap (blind rotate -> sample extract -> keyswitch) of a
batch of 4096 independent LWE ciphertexts per GPU, P-GATE parameters (n=630, k=1, N=1024,
PBS 2^7 x 3, KS 2^2 x 8), inputs resident in HBM before the timed region.  The default transform is
FFT64 (tfhe-rs's arithmetic: f64 negacyclic FFT external product over the native 2^64 torus,
pbs_fft.hip); --preset gate runs the same workload on the Goldilocks NTT transform (pbs_kernels.hip).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--cpu-sample S] [--preset gate_fft|gate|fhevm|fhevm_fft]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (one rank per GPU)

Multi-GPU: weak scaling.  Rank 0 generates the key set, uploads it to its GPU and broadcasts the
BSK/KSK once over RCCL (torch.distributed "nccl" backend = RCCL over xGMI); every rank then
bootstraps its own 4096-ciphertext batch with no data-path collective.  value = all ranks' PBS
divided by the MAX over ranks of the timed region.

--global-batch G: strong scaling instead (one batch of G PBS, contiguous slices of ~G/N per
rank; C4 = 65,536 -> 8,192 per GPU at N = 8); value = G x steps / max-over-ranks time.

The roofline figure is for the dominant kernel (blind rotation + fused sample extract), timed by HIP
events recorded by libtfhe_hip.so on the launch stream around every launch in the timed region.  Its
bound is the f64 VALU (see roofline()): frac = algorithmic f64 FLOP per PBS x batch / live kernel time /
78.6 TFLOP/s.  The VALU issue rate and the HBM traffic (and its ratio to the BSK + ciphertext floor) come
from the counter profile of THIS build (profiles/*_roofline.json with a matching tfhe_amd.source_id()).
The SURVEY §8d key-streaming byte model (61,952,960 B per PBS at r = 1) is reported as a labelled model only.

--preset fhevm runs the same protocol on the production fhEVM parameter set (P-FHEVM: n=918, k=1,
N=2048, PBS 2^23 x 1, KS 2^4 x 4, KS -> PBS; shortint messages m < 16, identity LUT) as a secondary
line; the headline metric is P-GATE.

cpu_baseline: rank 0 at N=1 only — the oracle's C restatement (oracle/, -O3, OpenMP, one PBS per
thread) on a bounded sample of the same inputs, same keys; the sample's outputs are also
compared bit-for-bit with the GPU's ("sample_bitexact").
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import tfhe_amd  # noqa: E402  (imports torch first: one HIP runtime per process)
from tfhe_amd.dist import broadcast_keys, rank_batch_seed  # noqa: E402

METRIC = "PBS/sec at TFHE 128-bit default (N=1024), batch=4096; 1/2/4/8 MI355X"
KEY_SEED = 0x7F4E0001
INPUT_SEED = 0xC0FFEE00
BR_BYTES_PER_PBS = 61_931_520 + 5_048 + 8_192 + 8_200   # blind-rotate kernel, key-streaming model (r = 1)
PBS_BYTES_PER_PBS = 103_303_024                           # whole PBS incl. KSK stream
# P-FHEVM blind rotate: BSK 918 x 2 x 2 x 2048 x 8 + small LWE in 919 x 8 + LUT 2048 x 8 + big LWE out 2049 x 8
BR_BYTES_PER_PBS_FHEVM = 60_162_048 + 7_352 + 16_384 + 16_392
FHEVM_MM = 16                                            # message 2 bits x carry 2 bits
C3_MASK = 0b10110010                                     # --config c3: bits bootstrapped with the NOT LUT
HBM_PEAK_GBS = 8000.0


def log(msg: str) -> None:
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


# Algorithmic f64 work of the FFT64 blind rotation per PBS, counted from the operation sequence the kernel and
# oracle/fft_oracle.c share (fma = 2 FLOP; complex multiply 6, complex add 2, radix-8 butterfly 56):
#   512-point DFT: forward 3 x 64 radix-8 + 2 x 64 x 7 twiddle cmul = 16,128; inverse (8 cmul in pass 2) 16,512;
#   N = 1024 forward = twist 512 cmul + DFT = 19,200, inverse = DFT + untwist = 19,584;
#   N = 2048 forward = twist 1024 cmul + 2 DFT + 512 radix-2 combines (10) = 43,520, inverse 44,288;
#   MAC = (k+1)l x (k+1) x N/2 complex fma (8).
#   P-GATE  (n=630, (k+1)l = 6): 6 x 19,200 + 2 x 19,584 + 6 x 2 x 512 x 8 = 203,520 FLOP per CMUX
#   P-FHEVM (n=918, (k+1)l = 2): 2 x 43,520 + 2 x 44,288 + 2 x 2 x 1024 x 8 = 208,384 FLOP per CMUX
FLOP_PER_PBS = {"gate_fft": 630 * 203_520, "fhevm_fft": 918 * 208_384}
F64_PEAK_TFLOPS = 78.6    # spec FP64 vector: 256 CUs x 4 SIMDs x 16 f64 lanes x 2 FLOP x 2.4 GHz
VALU_PEAK_GINST = 1024 * 2.4 / 4  # wave64 f64-rate VALU instructions / ns: 1024 SIMDs, 4 cycles each, 2.4 GHz


def profile_for(kernel: str, B: int):
    """Counter figures for `kernel` from the newest profiles/*_roofline.json whose source_id equals this
    tree's (tools/profile_round.sh -> tools/roofline_summary.py on the GPU box), measured at batch B.
    None when no profile of THIS build exists: a different build's counters are never reported."""
    import glob
    sid = tfhe_amd.source_id()
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_roofline.json")), reverse=True):
        d = json.load(open(f))
        if d.get("source_id") != sid or d.get("batch", 4096) != B:
            continue
        for k, v in d["kernels"].items():
            if k.split("<")[0].split("::")[-1] == kernel:
                return dict(v, source=os.path.relpath(f, ROOT), source_id=sid)
    return None


def roofline(preset: str, kernel: str, B: int, kernel_ms: float, br_bytes: int, floor_bytes: int) -> dict:
    """The dominant kernel's roofline: ALGORITHMIC f64 work against the FP64 vector peak.

    The blind rotation is bound by the f64 VALU, not by HBM: each BSK chunk is streamed once per workgroup into
    LDS and shared by its ciphertexts (and by resident workgroups through L2), so the measured HBM traffic is ~1 GB
    per 4096-PBS launch, not the 254 GB a key-streaming model (r = 1) would charge.  So
      frac = FLOP_PER_PBS x B / live kernel time / 78.6 TFLOP/s
    with FLOP_PER_PBS counted from the transforms' and MAC's operation sequence (fma = 2 FLOP) -- useful work only,
    independent of how many integer / move / conversion instructions the kernel spends around it.
    Reported beside it (same-build counter profile, profiles/*_roofline.json with this tree's source_id):
      valu_issue          SQ_INSTS_VALU x 4 cycles / (1024 SIMDs x 2.4 GHz x kernel time) -- an issue rate, not work
      traffic             HBM bytes per launch (FETCH_SIZE + WRITE_SIZE passes, gfx950-corrected)
      traffic_over_floor  traffic / (BSK + B x ciphertext bytes in and out): re-reads of the key per XCD and round
    Without a same-build profile those three are null."""
    prof = profile_for(kernel, B)
    s = kernel_ms * 1e-3
    flops = FLOP_PER_PBS.get(preset)
    out = {"kernel": kernel + " (+fused sample extract)", "kernel_ms": round(kernel_ms, 3)}
    if flops:
        tf = B * flops / s / 1e12
        out.update({"bound": "valu", "achieved": round(tf, 2), "peak": F64_PEAK_TFLOPS, "unit": "TFLOP/s",
                    "frac": round(tf / F64_PEAK_TFLOPS, 4), "flop_per_pbs": flops,
                    "model": "algorithmic f64 FLOP of the transforms + MAC per PBS (bench.py FLOP_PER_PBS, fma = 2) "
                             "x batch / live kernel time; peak = FP64 vector 256 CUs x 4 SIMDs x 16 lanes x 2 x 2.4 GHz"})
    else:  # the Goldilocks NTT engine: integer work, the VALU-issue figure is its roofline
        out.update({"bound": "valu", "achieved": None, "peak": VALU_PEAK_GINST, "unit": "G wave64-VALU-instr/s",
                    "frac": None})
    traffic = int(prof["hbm_bytes"]) if prof and prof.get("hbm_bytes") else None
    out["traffic"] = traffic
    out["traffic_floor_bytes"] = floor_bytes
    out["traffic_over_floor"] = round(traffic / floor_bytes, 2) if traffic else None
    if prof and prof.get("SQ_INSTS_VALU"):
        ginst = prof["SQ_INSTS_VALU"] / s / 1e9
        out["valu_issue"] = round(ginst / VALU_PEAK_GINST, 4)
        out["valu_insts_per_launch"] = int(prof["SQ_INSTS_VALU"])
        if not flops:
            out.update({"achieved": round(ginst, 1), "frac": out["valu_issue"]})
    else:
        out["valu_issue"] = None
    if traffic:
        gbs = traffic / s / 1e9
        out["hbm"] = {"achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
                      "traffic_per_pbs": round(traffic / B)}
    out["counters"] = ({"source": prof["source"], "source_id": prof["source_id"],
                        **{k: prof[k] for k in ("avg_ms", "SQ_WAIT_ANY_per_wave_cycle", "SQ_WAIT_INST_LDS_per_wave_cycle",
                                                "f64_share")
                           if k in prof}} if prof else
                       {"source": None, "note": f"no profiles/*_roofline.json for source_id {tfhe_amd.source_id()}"})
    # SURVEY 8(d)'s key-streaming model (r = 1: every PBS charged the whole BSK) -- a model, not a measurement
    out["hbm_model_r1"] = {"bytes_per_launch": B * br_bytes, "GBps_if_streamed": round(B * br_bytes / s / 1e9, 1),
                           "note": "model only: the BSK is shared through LDS/L2, see traffic"}
    return out


def host_cores() -> tuple:
    """CPUs this process may use: the affinity mask, capped by a cgroup CPU quota when one is set
    (a GPU box shows the whole machine's CPUs but grants a share)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    how = "sched_getaffinity"
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            lim = max(1, int(-(-int(q) // int(per))))
            if lim < n:
                n, how = lim, "cgroup cpu.max quota"
    except (OSError, ValueError):
        pass
    return n, how


def cpu_baseline(cts: np.ndarray, gpu_out: np.ndarray, sample: int, threads: int, preset: int = 0,
                 lut_host: np.ndarray = None, lut_idx: np.ndarray = None):
    """Oracle PBS on host cores over `sample` ciphertexts of the same batch (same keys)."""
    from oracle import oracle as O
    prm = O.params(preset)
    t = time.time()
    keys = O.Keys(prm, KEY_SEED)
    if prm.transform == 1:
        keys.bsk_fourier
    else:
        keys.bsk_ntt
    log(f"oracle keys in {time.time() - t:.1f}s")
    lut = O.lut_constant(1024, O.MU)[None] if lut_host is None else lut_host.reshape(-1, prm.N)
    sel = cts[:sample]
    idx = lut_idx[:sample] if lut_idx is not None else None
    w = max(1, threads // 4)
    O.pbs_batch(prm, keys, sel[:w], lut, idx[:w] if idx is not None else None, threads=threads)  # warm tables
    t = time.time()
    O.pbs_batch(prm, keys, sel[:1], lut, idx[:1] if idx is not None else None, threads=1)  # one PBS, one thread
    lat_ms = (time.time() - t) * 1e3
    # FFT64 presets: the timed leg is the SIMD port (oracle/fft_batch.c: the scalar restatement's operations on 8
    # AVX-512 or 4 AVX2 lanes, bit-identical to it -- tests/test_fft.py), the fairer CPU figure; one SIMD group on
    # one thread gives its per-PBS latency.  NTT presets: the scalar restatement, one PBS per thread.
    simd = prm.transform == 1
    simd_lat = None
    if simd:
        lanes = O.simd_lanes()
        O.pbs_batch_fft_simd(prm, keys, sel[:lanes], lut, idx[:lanes] if idx is not None else None, threads=1)
        t = time.time()
        O.pbs_batch_fft_simd(prm, keys, sel[:lanes], lut, idx[:lanes] if idx is not None else None, threads=1)
        simd_lat = (time.time() - t) * 1e3 / lanes
    t = time.time()
    if simd:
        ref = O.pbs_batch_fft_simd(prm, keys, sel, lut, idx, threads=threads)
    else:
        ref = O.pbs_batch(prm, keys, sel, lut, idx, threads=threads)
    dt = time.time() - t
    exact = bool(np.array_equal(ref, gpu_out[:sample]))
    digest = {"bitexact_pbs": sample, "gpu_sha256": hashlib.sha256(np.ascontiguousarray(gpu_out[:sample])).hexdigest(),
              "oracle_sha256": hashlib.sha256(np.ascontiguousarray(ref)).hexdigest()}
    return {
        "value": round(sample / dt, 3),
        "unit": "PBS/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{sample} PBS of the same {('P-GATE', 'P-FHEVM', 'P-GATE FFT64', 'P-FHEVM FFT64')[preset]} batch "
                  f"(first {sample} ciphertexts), "
                  + (f"SIMD C port (oracle/fft_batch.c: fft_oracle.c's operations on {lanes} f64 lanes, "
                     f"{'AVX-512F' if lanes == 8 else 'AVX2'}, {lanes} PBS per vector, bit-identical to the scalar "
                     f"restatement), OpenMP {threads} threads, one {lanes}-PBS group per thread, " if simd else
                     f"C oracle ({'oracle/fft_oracle.c' if prm.transform == 1 else 'oracle/tfhe_oracle.c'}, -O3 "
                     f"-march=x86-64-v3, OpenMP {threads} threads, one PBS per thread), ")
                  + f"{dt:.1f}s",
        "single_thread_ms_per_pbs": round(simd_lat if simd else lat_ms, 2),
        "scalar_oracle_single_thread_ms_per_pbs": round(lat_ms, 2),
    }, exact, digest


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=4096, help="PBS per GPU (weak scaling, the metric's mode)")
    ap.add_argument("--global-batch", type=int, default=0,
                    help="strong scaling: this many PBS in total, contiguous slices of ~G/N per rank (SURVEY 8e: "
                         "C4 = 65,536 -> 8,192 per GPU on 8 GPUs)")
    ap.add_argument("--cpu-sample", type=int, default=0, help="PBS in the CPU baseline sample (0 = auto)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL) on GPUs; gloo only for rehearsals")
    ap.add_argument("--preset", choices=["gate", "gate_fft", "fhevm", "fhevm_fft"], default="gate_fft",
                    help="gate_fft (default) = the BASELINE metric on the FFT64 transform (P-GATE, tfhe-rs's f64-FFT "
                         "external product over the native torus); gate = P-GATE on the Goldilocks NTT transform; "
                         "fhevm / fhevm_fft = production fhEVM parameters on the NTT / FFT64 transform (secondary line)")
    ap.add_argument("--config", choices=["metric", "c3"], default="metric",
                    help="metric (default) = BASELINE.json's headline PBS line; c3 = BASELINE.json configs[2]: --batch "
                         "FheUint8 ciphertexts, each bit bootstrapped with its own LUT (lut_index = bit position): "
                         "8 x batch PBS in ONE multi-LUT launch per step (P-GATE presets only)")
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal on a 1-GPU box: every rank uses device 0 (with --dist-backend gloo)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if args.same_device else int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    # a process group whenever a launcher set one up: N > 1, or torch.distributed.run with one rank (the 1-GPU
    # rehearsal of the RCCL path: key broadcast, barriers and the max-over-ranks all_reduce on a world-1 communicator)
    # (a launcher = torchrun's env: WORLD_SIZE plus LOCAL_RANK or TORCHELASTIC_RUN_ID; a scheduler that only exports
    # RANK / MASTER_ADDR does not turn a plain single-GPU run into an env:// rendezvous -- ADVICE r5)
    launched = "WORLD_SIZE" in os.environ and ("LOCAL_RANK" in os.environ or "TORCHELASTIC_RUN_ID" in os.environ)
    dist_on = world > 1 or launched
    if dist_on:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)

    fhevm = args.preset in ("fhevm", "fhevm_fft")
    fft = args.preset in ("gate_fft", "fhevm_fft")
    c3 = args.config == "c3"
    if c3 and fhevm:
        ap.error("--config c3 is the P-GATE FheUint8 workload (BASELINE.json configs[2]); use --preset gate_fft or gate")
    if c3 and args.global_batch:
        ap.error("--config c3 runs weak scaling only (--batch FheUint8 per GPU)")
    preset_id = {"gate": tfhe_amd.PRESET_GATE, "gate_fft": tfhe_amd.PRESET_GATE_FFT, "fhevm": tfhe_amd.PRESET_FHEVM,
                 "fhevm_fft": tfhe_amd.PRESET_FHEVM_FFT}[args.preset]
    params = tfhe_amd.Params.preset(preset_id)
    br_bytes = BR_BYTES_PER_PBS_FHEVM if fhevm else BR_BYTES_PER_PBS
    strong = args.global_batch > 0
    if strong:  # contiguous slice [lo, hi) of one global batch (SURVEY 8e partition)
        lo, hi = args.global_batch * rank // world, args.global_batch * (rank + 1) // world
        B = hi - lo
    else:
        lo, B = rank * args.batch, args.batch
    n_ct = B                 # ciphertexts of the workload (FheUint8 values under --config c3)
    if c3:                   # 8 bit-ciphertexts per FheUint8: the PBS batch of the one launch
        lo, B = 8 * lo, 8 * B

    # ---- key set: generated on rank 0, broadcast once over RCCL ---------------------------------
    t = time.time()
    bsk_len = tfhe_amd.lib().tfhe_hip_bsk_len(__import__("ctypes").byref(params))
    ksk_len = tfhe_amd.lib().tfhe_hip_ksk_len(__import__("ctypes").byref(params))
    if rank == 0:
        ck, sk = tfhe_amd.gen_keys(params, KEY_SEED)
        d_bsk = torch.from_numpy(sk.bsk.view(np.int64)).to(dev)
        d_ksk = torch.from_numpy(sk.ksk.view(np.int64)).to(dev)
        log(f"keygen {time.time() - t:.1f}s (BSK {sk.bsk.nbytes / 1e6:.1f} MB, KSK {sk.ksk.nbytes / 1e6:.1f} MB)")
    else:
        ck, _ = tfhe_amd.gen_keys(params, KEY_SEED, with_server_key=False)  # client key only (for checks)
        d_bsk = torch.empty(bsk_len, dtype=torch.int64, device=dev)
        d_ksk = torch.empty(ksk_len, dtype=torch.int64, device=dev)
    bcast_ms = 0.0
    if dist_on:
        dist.barrier()
        bcast_ms = broadcast_keys(d_bsk, d_ksk, src=0)
    eng = tfhe_amd.Engine(params, local)
    br_kernel = eng.br_kernel(B)  # the kernel the library's dispatch launches for this batch (profile matching)
    eng.load_keys_device(d_bsk, d_ksk)
    del d_bsk, d_ksk
    if fhevm:  # P-FHEVM server keys carry the modulus-switch noise-reduction zeros (10.6 MB, per rank)
        eng.load_ms_key(tfhe_amd.ms_zeros_keygen(params, KEY_SEED, ck.lwe_key))

    # ---- inputs: this rank's batch, encrypted on the host, resident in HBM ----------------------
    if strong:  # every rank draws the same global message vector and keeps its slice
        rng = np.random.default_rng(INPUT_SEED)
        gm = rng.integers(0, FHEVM_MM if fhevm else 2, args.global_batch)[lo:lo + B]
        rng = None
    else:
        rng = np.random.default_rng(rank_batch_seed(INPUT_SEED, rank))
    if fhevm:
        msgs = (gm if strong else rng.integers(0, FHEVM_MM, B)).astype(np.uint64)
        cts = ck.encrypt(msgs, FHEVM_MM, seed=INPUT_SEED + 1, stream0=lo)
        lut_host = eng.generate_accumulator(lambda m: m, FHEVM_MM)
    elif c3:
        # n_ct FheUint8 values, LSB first; bit j bootstrapped with LUT j (gate LUT or its negation, per C3_MASK):
        # the FheUint8.map_bits workload of tests/test_gpu_configs.py::test_c3_fheuint8_lut_eval_4096
        vals = (gm if strong else rng.integers(0, 256, n_ct)).astype(np.uint64)
        bits = ((vals[:, None] >> np.arange(8, dtype=np.uint64)[None, :]) & np.uint64(1)).astype(bool).reshape(-1)
        cts = ck.encrypt_bool(bits, seed=INPUT_SEED + 1, stream0=lo)
        gate = eng.gate_lut()
        inv = (np.uint64(0) - gate.astype(np.uint64)) % np.uint64(0xFFFFFFFF00000001)   # -1/8: NOT
        lut_host = np.stack([inv if (C3_MASK >> j) & 1 else gate for j in range(8)])
        lut_idx = np.tile(np.arange(8, dtype=np.uint32), n_ct)
    else:
        bits = (gm if strong else rng.integers(0, 2, B)).astype(bool)
        cts = ck.encrypt_bool(bits, seed=INPUT_SEED + 1, stream0=lo)
        lut_host = eng.gate_lut()
    d_in = torch.from_numpy(cts.view(np.int64)).to(dev)
    d_lut = torch.from_numpy(np.ascontiguousarray(lut_host).view(np.int64)).to(dev)
    d_idx = torch.from_numpy(lut_idx.view(np.int32)).to(dev) if c3 else None
    d_out = torch.empty_like(d_in)
    stream = torch.cuda.current_stream(dev)

    for _ in range(args.warmup):
        eng.pbs_async(d_in, d_lut, d_out, d_idx, stream=stream)
    torch.cuda.synchronize()

    eng.timing(True)
    eng.timing_reset()
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.pbs_async(d_in, d_lut, d_out, d_idx, stream=stream)
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    eng.timing(False)
    br_ms, br_n = eng.timing_stats(0)
    ks_ms, ks_n = eng.timing_stats(1)
    msr_ms, msr_n = eng.timing_stats(2)

    t_max = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if dist_on:
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
    elapsed_max = float(t_max.item())

    out = d_out.cpu().numpy().view(np.uint64)
    if fhevm:
        correct = bool(np.array_equal(ck.decrypt(out, FHEVM_MM), msgs))
    elif c3:
        got = ck.decrypt_bool(out).reshape(-1, 8).astype(np.uint64)
        correct = bool(np.array_equal((got << np.arange(8, dtype=np.uint64)[None, :]).sum(axis=1), vals ^ np.uint64(C3_MASK)))
    else:
        correct = bool(np.array_equal(ck.decrypt_bool(out), bits))
    ok = torch.tensor([1 if correct else 0], dtype=torch.int32, device=dev)
    if dist_on:
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)

    ms_per_step = elapsed_max * 1e3 / args.steps
    total_pbs = args.global_batch if strong else world * B
    value = total_pbs * args.steps / elapsed_max
    br_avg = br_ms / max(br_n, 1)

    pd = params.as_dict()
    bsk_bytes = pd["n"] * (pd["k"] + 1) * pd["pbs_level"] * (pd["k"] + 1) * pd["N"] * 8
    ksk_bytes = pd["k"] * pd["N"] * pd["ks_level"] * (pd["n"] + 1) * 8
    # ciphertexts in + out: small LWEs at P-GATE (PBS -> KS), big LWEs at P-FHEVM (KS -> PBS)
    io_bytes = 16 * ((pd["n"] + 1) if pd["order"] == 0 else (pd["k"] * pd["N"] + 1))
    result = None
    if rank == 0 and c3:
        result = {
            "metric": f"FheUint8 LUT evals/sec (8 PBS per ciphertext, one multi-LUT launch), batch={n_ct}",
            "value": round(world * n_ct * args.steps / elapsed_max, 1),
            "unit": "FheUint8/s",
            "pbs_per_s": round(value, 1),
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "f64" if fft else "u64",
            "data": "synthetic: uniform bytes, 8 ChaCha20-seeded gate-encoded bit LWEs each (key seed 0x7F4E0001); "
                    f"LUT j = NOT if bit j of {C3_MASK:#04x} else identity gate LUT (lut_index = bit position)",
            "config": {
                "workload": f"BASELINE.json configs[2]: FheUint8 LUT eval, {n_ct} FheUint8 x 8 per-bit LUTs = {B} P-GATE "
                            "PBS (blind rotate + sample extract + keyswitch) per GPU in one launch"
                            + (", FFT64 transform" if fft else ", NTT transform"),
                "batch_per_gpu": n_ct, "pbs_per_gpu": B, "params": params.as_dict(),
                "parallelism": f"batch-sharded x{world}",
            },
            "roofline": dict(roofline(args.preset, br_kernel, B, br_avg, br_bytes,
                                      bsk_bytes + B * 8 * ((pd["n"] + 1) + (pd["k"] * pd["N"] + 1))), launches=br_n),
            "keyswitch_ms": round(ks_ms / max(ks_n, 1), 3),
            "decrypt_ok": bool(ok.item()),
        }
        if world == 1 and not args.no_cpu:
            threads, how = host_cores()
            log(f"cpu baseline on {threads} host cores ({how})")
            sample = args.cpu_sample or (256 * threads if fft else 40 * threads)   # whole FheUint8 values: x 8
            sample = min(sample - sample % 8, B)
            cb, exact, digest = cpu_baseline(cts, out, sample, threads, preset_id, lut_host, lut_idx)
            cb["value_fheuint8_per_s"] = round(cb["value"] / 8, 3)
            result["cpu_baseline"] = cb
            result["sample_bitexact"] = exact
            result["bitexact_check"] = digest
        print(json.dumps(result), flush=True)
    elif rank == 0:
        result = {
            "metric": METRIC if not fhevm else f"PBS/sec at P-FHEVM (N=2048, KS->PBS), batch={B}",
            "value": round(value, 1),
            "unit": "PBS/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "f64" if fft else "u64",
            "data": ("synthetic: ChaCha20-seeded LWE encryptions of uniform bits (key seed 0x7F4E0001), gate LUT"
                     if not fhevm else "synthetic: ChaCha20-seeded shortint encryptions m < 16 under the big key "
                     "(key seed 0x7F4E0001), identity LUT"),
            "config": {
                "workload": ("P-GATE PBS (blind rotate + sample extract + keyswitch), n=630 k=1 N=1024, "
                             f"PBS 2^7x3, KS 2^2x8, batch {B} per GPU"
                             + (", FFT64 transform (f64 FFT over the 2^64 torus)" if fft else ", NTT transform (Z_p)"))
                            if not fhevm else
                            ("P-FHEVM PBS (keyswitch + blind rotate + sample extract), n=918 k=1 N=2048, "
                             f"PBS 2^23x1, KS 2^4x4, batch {B} per GPU"
                             + (", FFT64 transform (f64 FFT over the 2^64 torus)" if fft else ", NTT transform (Z_p)")),
                "batch_per_gpu": B,
                "global_batch": total_pbs,
                "params": params.as_dict(),
                "parallelism": f"batch-sharded x{world}, BSK/KSK RCCL broadcast once",
            },
            # the blind rotation's own floor: the BSK once + small LWEs in + extracted big LWEs out
            "roofline": dict(roofline(args.preset, br_kernel, B, br_avg, br_bytes,
                                      bsk_bytes + B * 8 * ((pd["n"] + 1) + (pd["k"] * pd["N"] + 1))),
                             # the reuse the kernel implements and the true minimum traffic
                             bsk_reuse=("latency kernel: one ciphertext per workgroup, key words from L2"
                                        if "lat" in br_kernel else
                                        "each CMUX's key words are read from L2 into registers once per workgroup and "
                                        "shared by its 2 ciphertexts (two workgroups per CU)"
                                        if args.preset == "fhevm_fft" else
                                        f"each BSK level-step chunk is streamed once per workgroup into LDS and shared "
                                        f"by its {dict(gate=8, gate_fft=2).get(args.preset, 4)} ciphertexts; resident workgroups share it through L2"),
                             min_traffic_bytes_per_pbs=round((bsk_bytes + ksk_bytes) / B + io_bytes),
                             launches=br_n),
            "keyswitch_ms": round(ks_ms / max(ks_n, 1), 3),
            "ms_noise_reduction_ms": round(msr_ms / msr_n, 3) if msr_n else None,
            "key_broadcast_ms": round(bcast_ms, 3),
            "dist": {"backend": dist.get_backend() if dist_on else None, "world_size": world},
            "decrypt_ok": bool(ok.item()),
        }
        if world == 1 and not args.no_cpu:
            threads, how = host_cores()
            log(f"cpu baseline on {threads} host cores ({how})")
            # ~10-20 s of CPU work: the oracle does ~3.5 PBS/s per thread on the NTT at P-GATE, ~23 on
            # FFT64, ~1.3 at P-FHEVM
            # FFT64: the whole 4096 batch at 16 threads (~11 s at P-GATE, ~15 s at P-FHEVM), so every output is
            # compared and the two SHA-256 digests cover the batch
            sample = args.cpu_sample or (max(256 * threads, 32) if fhevm and fft else max(16 * threads, 32) if fhevm
                                         else max(256 * threads, 64) if fft
                                         else max(40 * threads, 64))
            cb, exact, digest = cpu_baseline(cts, out, min(sample, B), threads, preset_id,
                                             lut_host if fhevm else None)
            result["cpu_baseline"] = cb
            result["sample_bitexact"] = exact
            result["bitexact_check"] = digest
        print(json.dumps(result), flush=True)
    if dist_on:
        dist.barrier()
        dist.destroy_process_group()
    eng.close()
    return 0 if bool(ok.item()) else 1


if __name__ == "__main__":
    sys.exit(main())
