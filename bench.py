#!/usr/bin/env python3
"""Benchmark of the MI355X turbo-decode hot path (BASELINE.json metric).

Workload (BASELINE.json configs[2], the configuration the metric is quoted
on): 16-QAM soft-LLR demap + DVB-RCS2 duo-binary turbo decode, N = 752 couples
(1504 info bits), rate 1/3, 8 iterations max-log-MAP.  One "step" = one pass
of the hot path over one batch of synthetic codewords already resident in
HBM: fused demap + de-puncture (k_demap_planes) followed by the fused turbo
decoder (k_turbo_decode), hard bits out.  Inputs are generated on the device
before the timed region by the counter-based generator (Philox info bits of
global codeword indices -> device encoder -> Gray 16-QAM -> complex AWGN).

Multi-GPU: one process per GPU.  `--gpus N` run as a plain `python bench.py`
spawns the N rank processes itself (the parent never touches the GPU); under
torchrun (WORLD_SIZE set) every process is already one rank.  Each rank
decodes its own contiguous range of global codewords (weak scaling, no
data-path collective); the barrier, the max-over-ranks time and the error
counters use torch.distributed (RCCL on the node).

Prints ONE JSON line on rank 0.
"""
import argparse
import hashlib
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

VALU_PEAK = 256 * 4 * 32 * 2.4e9     # lane-ops/s: 256 CU x 4 SIMD-32 x 2.4 GHz, a wave64 per 2 cycles (MI355X_MICROARCH.md)
HBM_PEAK = 8.0e12                    # B/s (spec)
SEED = 12345


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=1 << 20, help="codewords per GPU per step")
    ap.add_argument("--ebn0", type=float, default=2.0)
    ap.add_argument("--mod", default="16QAM")
    ap.add_argument("--n", type=int, default=752)
    ap.add_argument("--rate", default="1/3")
    ap.add_argument("--algo", default="max-log")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--fused", action="store_true", help="one launch (k_turbo_decode_syms, demap inside the "
                    "decoder waves) instead of k_demap_planes + k_turbo_decode (A/B; measured slower)")
    ap.add_argument("--overlap", action=argparse.BooleanOptionalAction, default=False,
                    help="demap of batch i+1 on its own handle / stream / plane buffer, free to fill the tail of "
                    "batch i's decode (DevicePipeline(overlap=True))")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL) on the node; gloo to rehearse "
                    "several ranks on one GPU together with --all-on-device0")
    ap.add_argument("--all-on-device0", action="store_true", help="every rank on GPU 0 (rehearsal on a 1-GPU box)")
    ap.add_argument("--rank-deadline", type=float, default=1800.0,
                    help="--gpus N without torchrun: kill every rank and exit non-zero after this many seconds")
    ap.add_argument("--dist-always", action="store_true",
                    help="initialise the process group (and time through its barrier / all-reduce) even for one "
                    "rank: exercises the RCCL path on a one-GPU box")
    ap.add_argument("--dist-timeout", type=float, default=300.0,
                    help="torch.distributed timeout (s) for rendezvous and collectives")
    a = ap.parse_args()
    if a.all_on_device0 and a.gpus > 1 and a.dist_backend == "nccl":
        ap.error("--all-on-device0 puts several ranks on one GPU, which RCCL cannot do: add --dist-backend gloo")
    return a


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_ranks(n, argv=None, deadline=None, script=None, poll=0.2):
    """`python bench.py --gpus N`: start N rank processes (one per GPU) and wait.

    Nothing in this parent initialises HIP; the children are fresh processes
    (never an exec of a process that touched the GPU).  Fail fast: when one rank
    exits non-zero the others are killed at once (they would wait at a barrier
    forever), and past `deadline` seconds every rank still running is killed and
    the return code is non-zero (124, as timeout(1)).  Returns the first
    non-zero exit code, or 0."""
    port = _free_port()
    argv = sys.argv[1:] if argv is None else argv
    script = os.path.abspath(__file__) if script is None else script
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, script, *argv], env=env))
    t_end = None if deadline is None else time.monotonic() + deadline
    rc = 0
    try:
        while procs:
            for p in list(procs):
                c = p.poll()
                if c is None:
                    continue
                procs.remove(p)
                if c != 0 and not rc:
                    rc = c
                    log(f"[spawn] a rank exited with {c}: stopping the other {len(procs)}")
                    for q in procs:
                        q.kill()
            if procs and t_end is not None and time.monotonic() > t_end:
                log(f"[spawn] deadline of {deadline:.0f}s passed with {len(procs)} rank(s) running: killing them")
                for q in procs:
                    q.kill()
                rc = rc or 124
                for q in procs:
                    q.wait()
                procs = []
            time.sleep(poll)
    finally:
        for p in procs:
            p.kill()
    return rc


def lib_sha256():
    from modulations_amd import _native
    with open(_native.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def measured_traffic(workload, kernel):
    """rocprof HBM bytes per codeword of `kernel` for this workload, only when
    profiles/traffic.json was measured on the exact library that is loaded."""
    tf = os.path.join(ROOT, "profiles", "traffic.json")
    if not os.path.exists(tf):
        return None, "no profiles/traffic.json"
    ent = json.load(open(tf)).get(kernel, {}).get(workload)
    if not ent:
        return None, "workload not profiled"
    from modulations_amd import _native
    from modulations_amd.build import build_info
    info = build_info(_native.LIB_PATH) or {}
    same_lib = ent.get("lib_sha256") == lib_sha256()
    same_src = ent.get("src_sha256") is not None and ent.get("src_sha256") == info.get("src_sha256")
    if not (same_lib or same_src):
        return None, "profiles/traffic.json was measured on another libtdec.so build (sources or binary)"
    return ent, None


def cpu_baseline(codec, syms_host, cons, bps, nv, div32, seconds):
    """The C oracle (bit-exact restatement, OpenMP over codewords) on a bounded
    sample of the same workload: demap + decode, on this host's cores."""
    from oracle import oracle as O
    from modulations_amd import tables as T
    t, _ = O.trellis()
    pm = T.puncture_matrix(codec.punct)
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    threads = min(threads, os.cpu_count() or threads)

    def run(rows, nthreads=threads):
        llr = np.stack([-O.demap(s, cons, bps, nv, div_f32=div32)[:codec.n_coded] for s in rows]).astype(np.float32)
        return O.decode_batch(llr, codec.N, codec.punct["period"], pm, codec.iterations, codec.perm,
                              codec.inv_perm, t, algo=codec.algo, nthreads=nthreads)

    t0 = time.perf_counter()
    run(syms_host[:threads])
    per = (time.perf_counter() - t0) / threads             # s per codeword per thread (calibration)
    n = int(max(threads, min(len(syms_host), seconds * threads / max(per, 1e-6))))
    t0 = time.perf_counter()
    run(syms_host[:n])
    dt = time.perf_counter() - t0
    n1 = int(max(1, min(len(syms_host), 3.0 / max(per * threads, 1e-6))))   # ~3 s on one core
    t0 = time.perf_counter()
    run(syms_host[:n1], 1)
    dt1 = time.perf_counter() - t0
    out = {"value": n / dt, "unit": "codewords/s", "cores": threads, "kind": "port",
           "sample": f"{n} codewords of the same workload (oracle demap + decode, OpenMP over codewords on "
                     f"{threads} threads), {dt:.1f} s; single core: {n1} codewords, {dt1:.1f} s",
           "info_bits_per_s": n * codec.k_info / dt, "single_core_value": n1 / dt1}
    cal = os.path.join(ROOT, "profiles", "cpu_calibration.json")
    if os.path.exists(cal):
        c = json.load(open(cal))
        out["numba_ratio"] = c["ratio_1core"]
        out["numba_calibration"] = (f"the C restatement decodes {c['oracle_1t_cw_per_s']:.0f} cw/s on one core of the "
                                    f"survey's container vs the reference's numba machine code at "
                                    f"{c['numba_1core_cw_per_s']:.0f} cw/s there (SURVEY.md §6; N=752 r=1/3 decode "
                                    f"only): ratio {c['ratio_1core']:.2f} (profiles/cpu_calibration.json)")
    return out


def host_api(codec, llr_rows, hb, dev):
    """The host-pointer drop-in boundary, PCIe included (informational, never `value`):
    DVBRCS2_Turbo.decode_batch over numpy buffers (pageable, then page-locked
    host_buffer()s), and the single-call latency of the reference's own harness
    pattern: DVBRCS2_Turbo(752, '1/2').decode(llr) once per frame (test.py:81), and
    one bcjr_max_log_map call (N=752)."""
    from modulations_amd import dvb_rcs2_turbo as M
    llr_h = np.ascontiguousarray(np.tile(llr_rows, (-(-hb // len(llr_rows)), 1))[:hb])
    nbytes = hb * (llr_h.shape[1] * 4 + codec.k_info * 4)
    res = {"unit": "codewords/s", "batch": hb, "bytes_per_codeword": nbytes / hb}
    codec.decode_batch(llr_h)                 # steady state: staging buffers already sized
    t0 = time.perf_counter()
    codec.decode_batch(llr_h)
    dt = time.perf_counter() - t0
    res.update({"value": hb / dt, "pcie_GBps": nbytes / dt / 1e9,
                "path": "DVBRCS2_Turbo.decode_batch(numpy f32 [B, n_coded], pageable; the bench's own noisy LLRs, "
                        "1024 distinct rows tiled) -> numpy int32, H2D + depuncture + decode + D2H in chunks of "
                        "65536 on three streams (upload / decode / download)"})
    pin_llr = M.DVBRCS2_Turbo.host_buffer(llr_h.shape, np.float32)
    pin_llr[...] = llr_h
    pin_bits = M.DVBRCS2_Turbo.host_buffer((hb, codec.k_info), np.int32)
    codec.decode_batch(pin_llr, out=pin_bits)
    t0 = time.perf_counter()
    codec.decode_batch(pin_llr, out=pin_bits)
    dt = time.perf_counter() - t0
    res["pinned"] = {"value": hb / dt, "pcie_GBps": nbytes / dt / 1e9,
                     "path": "the same call over page-locked host_buffer()s (tdec_host_alloc) for the LLRs and the bits",
                     "same_bits": bool(np.array_equal(pin_bits[:4096], codec.decode_batch(llr_h[:4096])))}
    # single-call latency: test.py's pattern (one decode() per frame, test.py:81) and one
    # bcjr_max_log_map call, at each BASELINE block size.  Reference: numba on one core
    # (SURVEY §6 / BASELINE.md §2): decode 1.22 / 3.89 / 12.30 ms (r=1/3; 11.78 at 752 r=1/2);
    # SISO 0.493 ms measured at N=752, 0.058 / 0.143 ms at N=48 / 212 derived as decode time
    # x SISO share / 16 (76 % / 59 %).
    ref_dec = {(48, "1/3"): 1.22, (212, "1/3"): 3.89, (752, "1/3"): 12.30, (752, "1/2"): 11.78}
    ref_siso = {48: 0.058, 212: 0.143, 752: 0.493}
    rng = np.random.default_rng(3)
    sc = {}
    for (n, rate), ref in ref_dec.items():
        cc = M.DVBRCS2_Turbo(n, rate, 8, device=dev)
        frames = []
        for _ in range(51):
            b = rng.integers(0, 2, cc.k_info)
            frames.append(((1 - 2.0 * cc.encode(b)) * 2.0 + rng.standard_normal(cc.n_coded) * 1.5).astype(np.float32))
        cc.decode(frames[0])                      # handle creation and workspace reserve, once
        ts = []
        for f in frames[1:]:
            t0 = time.perf_counter()
            cc.decode(f)
            ts.append(time.perf_counter() - t0)
        sc[f"decode_{n}_r{rate.replace('/', '')}"] = {"ms": float(np.median(ts) * 1e3), "min_ms": float(np.min(ts) * 1e3),
                                                    "reference_ms": ref, "x_reference": ref / float(np.median(ts) * 1e3)}
    t = M._std_tables()[:5]   # next_state, out_W, out_Y, prev_state, prev_input
    for n, ref in ref_siso.items():
        Lc = (rng.standard_normal((4, n)) * 3).astype(np.float32)
        La = rng.standard_normal((2, n)) * 5
        M.bcjr_max_log_map(*Lc, *La, *t, n, 0.7)
        ts2 = []
        for _ in range(200):
            t0 = time.perf_counter()
            M.bcjr_max_log_map(*Lc, *La, *t, n, 0.7)
            ts2.append(time.perf_counter() - t0)
        sc[f"bcjr_max_log_map_{n}"] = {"ms": float(np.median(ts2) * 1e3), "min_ms": float(np.min(ts2) * 1e3),
                                       "reference_ms": ref, "x_reference": ref / float(np.median(ts2) * 1e3)}
    sc["path"] = ("DVBRCS2_Turbo(N, rate).decode(llr) per frame as test.py:81 (median of 50 noisy frames); "
                  "bcjr_max_log_map(...) per call, f32 Lc (median of 200); reference: numba, one core, SURVEY §6")
    res["single_call_ms"] = sc
    return res


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus, deadline=args.rank_deadline))

    import torch
    from modulations_amd import demap as D
    from modulations_amd import dvb_rcs2_turbo as M
    from modulations_amd import sharding as Sh
    from modulations_amd.workload import DevicePipeline, count_errors, make_symbols

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1 or args.dist_always
    tdist = None
    dev_idx = 0 if args.all_on_device0 else local
    torch.cuda.set_device(dev_idx)
    if dist:
        import datetime
        import torch.distributed as tdist
        to = datetime.timedelta(seconds=args.dist_timeout)
        if args.dist_backend == "nccl":
            tdist.init_process_group("nccl", device_id=torch.device("cuda", dev_idx), timeout=to)
        else:
            tdist.init_process_group(args.dist_backend, timeout=to)
    device = torch.device("cuda", dev_idx)

    codec = M.DVBRCS2_Turbo(args.n, args.rate, 8, algo=args.algo, device=device.index)
    if dist:   # every rank must decode with the same de-interleaver (sharding.check_same_interleaver)
        Sh.check_same_interleaver(codec.inv_perm, tdist, device if args.dist_backend == "nccl" else torch.device("cpu"))
    bps = D.MODULATIONS[args.mod]["bps"]
    cons = D.constellation(args.mod)
    B = args.batch
    cw0 = rank * B                                   # this rank's global codewords: [rank*B, (rank+1)*B)
    t0 = time.time()
    # decoder workspace and planes first, into unfragmented HBM (placement)
    pipe = DevicePipeline(codec, args.mod, B, device, fused=args.fused, overlap=args.overlap)
    _, syms, n0 = make_symbols(codec, B, args.mod, args.ebn0, SEED, device, cw0=cw0, want_info=False)
    syms_ready = torch.cuda.Event()
    syms_ready.record()
    S = syms.shape[1]
    nv = np.float64(n0)
    f64, div32, nve = D.demap_mode(np.complex64, cons.dtype, nv)
    bits = pipe.bits
    torch.cuda.synchronize()
    log(f"[rank {rank}] workload ready: {B} codewords x {S} symbols in {time.time() - t0:.1f}s")

    stream = torch.cuda.current_stream()

    def step(ev=None):
        pipe.run(syms, nv, stream=stream, events=ev, syms_ready=syms_ready)

    for i in range(args.warmup):
        step()
        torch.cuda.synchronize()
        log(f"[rank {rank}] warmup {i + 1}/{args.warmup}")

    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if dist:
        tdist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for i in range(args.steps):
        step(evs[i])
    torch.cuda.synchronize()
    if dist:
        tdist.barrier()
    elapsed = time.perf_counter() - t_start
    # k_turbo_decode launch duration: events recorded on the stream the kernel runs on
    dec_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    log(f"[rank {rank}] timed {args.steps} steps in {elapsed:.3f}s, decode kernel {dec_ms:.2f} ms/launch")

    # error counters (not timed): info-bit errors, frame errors, codewords, against the generator's bits
    errs = count_errors(codec, bits, SEED, cw0=cw0)
    red_dev = device if (not dist or args.dist_backend == "nccl") else torch.device("cpu")
    cnt = torch.tensor([int(errs.sum(dtype=torch.int64)), int((errs > 0).sum()), B], dtype=torch.int64,
                       device=red_dev)
    tmax = torch.tensor([elapsed], dtype=torch.float64, device=red_dev)
    dmax = torch.tensor([dec_ms], dtype=torch.float64, device=red_dev)
    Sh.reduce_counters(cnt, tdist)
    Sh.reduce_max(tmax, tdist)
    Sh.reduce_max(dmax, tdist)
    elapsed = float(tmax)
    total_cw = B * world * args.steps
    value = total_cw / elapsed

    if rank == 0:
        wl = (f"{args.mod} soft-LLR demap + DVB-RCS2 turbo N={args.n} couples ({2 * args.n} info bits) "
              f"r={args.rate}, 8 it {args.algo}-MAP")
        kname = "k_turbo_decode_logmap" if codec.algo else "k_turbo_decode"
        ops = 2 * codec.iterations * codec.N * 768            # SURVEY §8(d) lane-op count per codeword
        valu_achieved = B * ops / (dec_ms * 1e-3)              # per GPU: this rank's launch
        alg_bytes = B * (4 * codec.n_coded + 4 * codec.k_info)  # f32 LLRs in + int32 bits out per codeword
        tr, why = measured_traffic(wl, kname)
        traffic = tr["hbm_bytes_per_codeword"] * B if tr else None
        out = {
            "metric": "codewords/sec + info-bits/sec, N=1504 r=1/3 8-iter max-log-MAP @1/2/4/8 GPU",
            "value": value,
            "unit": "codewords/s",
            "info_bits_per_s": value * codec.k_info,
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32 (recursions) / f64 (branch sums, extrinsic)",
            "data": "synthetic (device counter-based generator: Philox info bits -> encoder -> Gray "
                    f"{args.mod} -> AWGN)",
            "config": {"workload": wl, "codewords_per_gpu_per_step": B, "ebn0_db": args.ebn0,
                       "parallelism": f"codeword shards x{world}"},
            "roofline": {
                "bound": "valu", "kernel": kname,
                "achieved": valu_achieved / 1e12, "peak": VALU_PEAK / 1e12, "unit": "T lane-op/s",
                "frac": valu_achieved / VALU_PEAK,
                "traffic": traffic,
                "note": "SURVEY §8(d): the recursions are VALU issue work, W = 2*I*N*768 f32 lane-ops per codeword "
                        f"({ops}); achieved = W x codewords per launch / k_turbo_decode launch time (HIP events "
                        "on its stream); peak = 256 CU x 4 SIMD-32 x 2.4 GHz (a wave64 VALU op per 2 cycles). "
                        "traffic = rocprof-measured HBM bytes per launch (profiles/traffic.json, used only when "
                        "stamped with the sha256 of the loaded libtdec.so)",
            },
            "hbm": {
                "algorithmic_GBps": alg_bytes / (dec_ms * 1e-3) / 1e9, "peak_GBps": HBM_PEAK / 1e9,
                "algorithmic_frac": alg_bytes / (dec_ms * 1e-3) / HBM_PEAK,
                "algorithmic_bytes_per_codeword": alg_bytes / B,
                "measured_bytes_per_codeword": tr["hbm_bytes_per_codeword"] if tr else None,
                "measured_GBps": (traffic / (dec_ms * 1e-3) / 1e9) if traffic else None,
                "measured_source": tr.get("source") if tr else why,
            },
            "decode_kernel_ms": dec_ms,
            "decode_kernel_ms_max_over_ranks": float(dmax),
            "ber": {"bit_errors": int(cnt[0]), "frame_errors": int(cnt[1]), "codewords": int(cnt[2]),
                    "info_ber": int(cnt[0]) / (int(cnt[2]) * codec.k_info)},
        }
        if world == 1 and not args.no_cpu:
            syms_host = syms[:min(B, 80000)].cpu().numpy()
            from oracle import oracle as O
            llr_rows = np.stack([-O.demap(s, cons, bps, nve, div_f32=div32)[:codec.n_coded]
                                 for s in syms_host[:1024]]).astype(np.float32)
            out["host_api"] = host_api(codec, llr_rows, min(B, 262144), device.index)
            log("[rank 0] timing the CPU baseline (oracle) ...")
            out["cpu_baseline"] = cpu_baseline(codec, syms_host, cons, bps, nve, div32, args.cpu_seconds)
            # parity spot-check of the timed GPU output against the oracle on the same sample
            from modulations_amd import tables as T
            t, _ = O.trellis()
            if codec.algo:   # the build-defined log-MAP: pin the oracle to this device's primitives
                O.set_trans(M.capture_trans_tables(device.index))
            chk = 64
            rb = O.decode_batch(llr_rows[:chk], codec.N, codec.punct["period"], T.puncture_matrix(codec.punct), 8,
                                codec.perm, codec.inv_perm, t, algo=codec.algo)
            out["parity_spot_check"] = bool(np.array_equal(bits[:chk].cpu().numpy(), rb))
        print(json.dumps(out), flush=True)
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
