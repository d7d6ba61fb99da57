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

The roofline figure is for the dominant kernel (blind rotation + fused sample extract): HIP
events recorded by libtfhe_hip.so on the launch stream around every launch in the timed region;
algorithmic bytes per PBS = 61,952,960 (BSK 61,931,520 + LWE in 5,048 + LUT 8,192 + extracted
LWE 8,200: SURVEY §8d), peak 8.0 TB/s (MI355X HBM3E, MI355X_MICROARCH.md).

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
HBM_PEAK_GBS = 8000.0


def log(msg: str) -> None:
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def pmc_traffic(B: int, kernel: str = "blind_rotate_kernel"):
    """HBM bytes per blind-rotate launch from the committed rocprofv3 PMC passes
    (profiles/*_pmc_blind_rotate.json, produced by tools/pmc_summary.py for this same command), or None."""
    import glob
    if B != 4096:
        return None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_blind_rotate.json")), reverse=True):
        for k, v in json.load(open(f)).items():  # the newest pass that profiled this kernel
            if k.split("<")[0].endswith("::" + kernel):
                return round(v["hbm_bytes_per_launch"])
    return None


def valu_profile(B: int, kernel_ms: float, kernel: str = "blind_rotate_kernel"):
    """VALU roofline of the blind-rotate kernel from the committed SQ counter pass
    (profiles/*_pmc_sq.csv: rocprofv3 --pmc SQ_INSTS_VALU ... of this bench at B = 4096): wave64 VALU
    instructions per launch (scaled per PBS to B) x 4 cycles on a 16-lane SIMD, over the SIMD-cycles of
    the measured launch (1024 SIMDs at 2.4 GHz, MI355X_MICROARCH.md)."""
    import csv
    import glob
    vals, src = [], None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_sq.csv")), reverse=True):
        vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if r["Counter_Name"] == "SQ_INSTS_VALU"
                and r["Kernel_Name"].split("(")[0].split("<")[0].endswith("::" + kernel)]
        if vals:  # the newest pass that profiled this kernel
            src = f
            break
    if not vals:
        return None
    insts = sum(vals) / len(vals) / 4096 * B
    frac = insts * 4 / (1024 * 2.4e9 * kernel_ms * 1e-3)
    out = {"bound": "valu", "insts_per_launch": round(insts), "insts_per_pbs": round(insts / B),
           "issue_frac": round(frac, 3), "model": "4 cycles per wave64 VALU instruction per SIMD, 1024 SIMDs, 2.4 GHz",
           "source": os.path.relpath(src, ROOT)}
    # the same instructions priced at the f64 rate measured on this hardware (independent v_fma_f64 /
    # v_add_f64 chains, 2 waves per SIMD: tools/microbench/f64_rates.hip -> profiles/r01_f64_rates.txt)
    rates = os.path.join(ROOT, "profiles", "r01_f64_rates.txt")
    if "fft" in kernel and os.path.exists(rates):
        cyc = [float(l.split()[3]) for l in open(rates) if l.split() and l.split()[0] in ("v_fma_f64", "v_add_f64")]
        if cyc:
            c = sum(cyc) / len(cyc)
            out["measured_rate_frac"] = round(insts * c / (1024 * 2.4e9 * kernel_ms * 1e-3), 3)
            out["measured_rate_model"] = f"{c:.2f} nominal cycles per f64 wave64 instruction (microbenchmark)"
    return out


def cpu_baseline(cts: np.ndarray, gpu_out: np.ndarray, sample: int, threads: int, preset: int = 0,
                 lut_host: np.ndarray = None):
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
    lut = O.lut_constant(1024, O.MU)[None] if lut_host is None else lut_host[None]
    sel = cts[:sample]
    O.pbs_batch(prm, keys, sel[: max(1, threads // 4)], lut, threads=threads)  # warm tables
    t = time.time()
    O.pbs_batch(prm, keys, sel[:1], lut, threads=1)  # single-thread latency of one PBS
    lat_ms = (time.time() - t) * 1e3
    t = time.time()
    ref = O.pbs_batch(prm, keys, sel, lut, threads=threads)
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
                  f"(first {sample} ciphertexts), C oracle "
                  f"({'oracle/fft_oracle.c' if prm.transform == 1 else 'oracle/tfhe_oracle.c'}, -O3 "
                  f"-march=x86-64-v3, OpenMP {threads} threads, one PBS per thread), "
                  f"{dt:.1f}s",
        "single_thread_ms_per_pbs": round(lat_ms, 2),
    }, exact, digest


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--cpu-sample", type=int, default=0, help="PBS in the CPU baseline sample (0 = auto)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL) on GPUs; gloo only for rehearsals")
    ap.add_argument("--preset", choices=["gate", "gate_fft", "fhevm", "fhevm_fft"], default="gate_fft",
                    help="gate_fft (default) = the BASELINE metric on the FFT64 transform (P-GATE, tfhe-rs's f64-FFT "
                         "external product over the native torus); gate = P-GATE on the Goldilocks NTT transform; "
                         "fhevm / fhevm_fft = production fhEVM parameters on the NTT / FFT64 transform (secondary line)")
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
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)

    fhevm = args.preset in ("fhevm", "fhevm_fft")
    fft = args.preset in ("gate_fft", "fhevm_fft")
    preset_id = {"gate": tfhe_amd.PRESET_GATE, "gate_fft": tfhe_amd.PRESET_GATE_FFT, "fhevm": tfhe_amd.PRESET_FHEVM,
                 "fhevm_fft": tfhe_amd.PRESET_FHEVM_FFT}[args.preset]
    params = tfhe_amd.Params.preset(preset_id)
    br_kernel = {"gate": "blind_rotate_kernel", "gate_fft": "blind_rotate_fft_kernel",
                 "fhevm": "blind_rotate2048_kernel", "fhevm_fft": "blind_rotate_fft2k_kernel"}[args.preset]
    br_bytes = BR_BYTES_PER_PBS_FHEVM if fhevm else BR_BYTES_PER_PBS
    B = args.batch

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
    if world > 1:
        dist.barrier()
        bcast_ms = broadcast_keys(d_bsk, d_ksk, src=0)
    eng = tfhe_amd.Engine(params, local)
    eng.load_keys_device(d_bsk, d_ksk)
    del d_bsk, d_ksk
    if fhevm:  # P-FHEVM server keys carry the modulus-switch noise-reduction zeros (10.6 MB, per rank)
        eng.load_ms_key(tfhe_amd.ms_zeros_keygen(params, KEY_SEED, ck.lwe_key))

    # ---- inputs: this rank's batch, encrypted on the host, resident in HBM ----------------------
    rng = np.random.default_rng(rank_batch_seed(INPUT_SEED, rank))
    if fhevm:
        msgs = rng.integers(0, FHEVM_MM, B).astype(np.uint64)
        cts = ck.encrypt(msgs, FHEVM_MM, seed=INPUT_SEED + 1, stream0=rank * B)
        lut_host = eng.generate_accumulator(lambda m: m, FHEVM_MM)
    else:
        bits = rng.integers(0, 2, B).astype(bool)
        cts = ck.encrypt_bool(bits, seed=INPUT_SEED + 1, stream0=rank * B)
        lut_host = eng.gate_lut()
    d_in = torch.from_numpy(cts.view(np.int64)).to(dev)
    d_lut = torch.from_numpy(lut_host.view(np.int64)).to(dev)
    d_out = torch.empty_like(d_in)
    stream = torch.cuda.current_stream(dev)

    for _ in range(args.warmup):
        eng.pbs_async(d_in, d_lut, d_out, stream=stream)
    torch.cuda.synchronize()

    eng.timing(True)
    eng.timing_reset()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.pbs_async(d_in, d_lut, d_out, stream=stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    eng.timing(False)
    br_ms, br_n = eng.timing_stats(0)
    ks_ms, ks_n = eng.timing_stats(1)
    msr_ms, msr_n = eng.timing_stats(2)

    t_max = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
    elapsed_max = float(t_max.item())

    out = d_out.cpu().numpy().view(np.uint64)
    if fhevm:
        correct = bool(np.array_equal(ck.decrypt(out, FHEVM_MM), msgs))
    else:
        correct = bool(np.array_equal(ck.decrypt_bool(out), bits))
    ok = torch.tensor([1 if correct else 0], dtype=torch.int32, device=dev)
    if world > 1:
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)

    ms_per_step = elapsed_max * 1e3 / args.steps
    value = world * B * args.steps / elapsed_max
    br_avg = br_ms / max(br_n, 1)
    achieved = B * br_bytes / (br_avg * 1e-3) / 1e9

    pd = params.as_dict()
    bsk_bytes = pd["n"] * (pd["k"] + 1) * pd["pbs_level"] * (pd["k"] + 1) * pd["N"] * 8
    ksk_bytes = pd["k"] * pd["N"] * pd["ks_level"] * (pd["n"] + 1) * 8
    # ciphertexts in + out: small LWEs at P-GATE (PBS -> KS), big LWEs at P-FHEVM (KS -> PBS)
    io_bytes = 16 * ((pd["n"] + 1) if pd["order"] == 0 else (pd["k"] * pd["N"] + 1))
    result = None
    if rank == 0:
        result = {
            "metric": METRIC if not fhevm else f"PBS/sec at P-FHEVM (N=2048, KS->PBS), batch={B}",
            "value": round(value, 1),
            "unit": "PBS/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
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
                "params": params.as_dict(),
                "parallelism": f"batch-sharded x{world}, BSK/KSK RCCL broadcast once",
            },
            "roofline": {
                "bound": "hbm",
                "kernel": br_kernel + " (+fused sample extract)",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": pmc_traffic(B, br_kernel),
                "bytes_per_launch": B * br_bytes,
                "kernel_ms": round(br_avg, 3),
                "launches": br_n,
                # the reuse the kernel implements and the true minimum traffic
                "bsk_reuse": (f"each BSK level-step chunk is streamed once per workgroup into LDS and shared by its "
                              f"{8 if not (fhevm and fft) else 4} ciphertexts; resident workgroups share it through L2"),
                "min_traffic_bytes_per_pbs": round((bsk_bytes + ksk_bytes) / B + io_bytes),
            },
            "valu_roofline": valu_profile(B, br_avg, br_kernel),
            "keyswitch_ms": round(ks_ms / max(ks_n, 1), 3),
            "ms_noise_reduction_ms": round(msr_ms / msr_n, 3) if msr_n else None,
            "key_broadcast_ms": round(bcast_ms, 3),
            "decrypt_ok": bool(ok.item()),
        }
        if world == 1 and not args.no_cpu:
            threads = min(os.cpu_count() or 1, int(os.environ.get("OMP_NUM_THREADS", "16") or 16))
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
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    eng.close()
    return 0 if bool(ok.item()) else 1


if __name__ == "__main__":
    sys.exit(main())
