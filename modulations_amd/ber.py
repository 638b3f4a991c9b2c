"""Coded-BER Monte-Carlo sweep on MI355X (BASELINE.json configs[3]/[4]):
Eb/N0 points x codewords, sharded over GPUs with torchrun, resumable.

  python -m modulations_amd.ber --mod 256QAM --n 752 --rate 1/3 --ebn0=-2:10:1 \
      --codewords 10000000 --out ber_256qam.json
  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m modulations_amd.ber ...

Each rank owns a contiguous range of global codeword indices per point
(sharding.shard_range) and generates it on its own device with the
counter-based generator (seed per point, counter = global codeword index: the
data, and so the counters, are the same for any world size or batch size),
runs the fused demap + decode, and counts bit / frame errors on the device;
only those int64 counters are all-reduced.  Finished points are written to
--out after every point, and a rerun skips them (checkpoint / resume, SURVEY
§5).  The file records the sweep's configuration and the generator version;
a rerun into it with any other configuration (modulation, block size, rate,
algorithm, iterations, interleaver, codewords per point, base seed) or
generator is refused instead of mixing two data streams, and each point's
generator key is derived from its Eb/N0 value (not its index in --ebn0), so a
resumed sweep over a different grid regenerates exactly the same data.
"""
from __future__ import annotations

import argparse
import json
import os
import time

import numpy as np


GENERATOR = "philox4x32-10/global-codeword-index/v2"   # workload.make_symbols' stream; bump on any change


def ebn0_seed(base_seed, ebn0_db):
    """Generator key of the point at `ebn0_db`: the base seed and the Eb/N0
    value in milli-dB, so the key does not depend on the point's position in
    the sweep grid (64-bit, as the device generator takes it)."""
    return (int(base_seed) * 1_000_003 + int(round(float(ebn0_db) * 1000)) * 7919) & 0xFFFFFFFFFFFFFFFF


def sweep_config(a, inv_perm=None):
    """What a results file is keyed on (argparse namespace -> dict), including the
    digest of the inverse interleaver actually used (sharding.interleaver_digest:
    the reference's default differs between numpy builds)."""
    from .sharding import interleaver_digest
    cfg = {"generator": GENERATOR, "mod": a.mod, "n_couples": int(a.n), "rate": a.rate, "algo": a.algo,
           "iterations": int(a.iterations), "interleaver": a.interleaver, "codewords": int(a.codewords),
           "seed": int(a.seed)}
    if inv_perm is not None:
        cfg["inv_perm_digest"] = interleaver_digest(inv_perm)
    return cfg


def load_resume(path, cfg):
    """Finished points of `path` for the sweep configuration `cfg`:
    {ebn0_db: record}.  A missing file is an empty sweep; a file written for
    another configuration or generator (or in the old unkeyed list format)
    raises ValueError rather than silently merging points of two streams."""
    if not path or not os.path.exists(path):
        return {}
    with open(path) as f:
        doc = json.load(f)
    if not isinstance(doc, dict) or "config" not in doc:
        raise ValueError(f"{path}: results without a sweep configuration (old format); use another --out")
    if doc["config"] != cfg:
        diff = {k: (doc["config"].get(k), cfg.get(k)) for k in set(doc["config"]) | set(cfg)
                if doc["config"].get(k) != cfg.get(k)}
        raise ValueError(f"{path}: written for another sweep configuration {diff} (file, this run); use another --out")
    return {float(r["ebn0_db"]): r for r in doc["points"]}


def save_results(path, cfg, results):
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump({"config": cfg, "points": sorted(results, key=lambda r: r["ebn0_db"])}, f, indent=1)
    os.replace(tmp, path)


def parse_points(spec):
    if ":" in spec:
        a, b, s = (float(x) for x in spec.split(":"))
        return [round(a + i * s, 6) for i in range(int(round((b - a) / s)) + 1)]
    return [float(x) for x in spec.split(",")]


def run_point(pipe, codec, mod, ebn0, start, count, batch, seed, device, times=None):
    """Bit errors, frame errors and codewords of global codewords
    [start, start + count) at one Eb/N0 point.  The data of codeword g is a
    counter-based stream of (seed, g) (workload.make_symbols), so the counters
    do not depend on the batch size or on how the job is sharded.  times (a list,
    optional): per batch, (demap + decode ms, decode ms) from HIP events on the
    pipeline's stream -- the bench's timed step, without the generator and the
    error counting."""
    import torch
    from . import sharding as S
    from .workload import count_errors, make_symbols
    cnt = torch.zeros(3, dtype=torch.int64, device=device)
    ev = []
    for off, n in S.batches(count, batch):
        _, syms, n0 = make_symbols(codec, n, mod, ebn0, seed, device, cw0=start + off, want_info=False)
        e3 = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        e3[0].record()
        bits = pipe.run(syms, n0, events=e3[1:])[:n]
        ev.append(e3)
        e = count_errors(codec, bits, seed, cw0=start + off)
        cnt += torch.stack([e.sum(dtype=torch.int64), (e > 0).sum(), torch.tensor(n, device=device)]).to(torch.int64)
    if times is not None:
        torch.cuda.synchronize()
        times += [(a.elapsed_time(c), b.elapsed_time(c)) for a, b, c in ev]
    return cnt


def main(argv=None):
    import torch
    import torch.distributed as dist
    from . import dvb_rcs2_turbo as M
    from . import sharding as S
    from .workload import DevicePipeline

    ap = argparse.ArgumentParser()
    ap.add_argument("--mod", default="256QAM")
    ap.add_argument("--n", "--couples", dest="n", type=int, default=752)
    ap.add_argument("--rate", default="1/3")
    ap.add_argument("--algo", default="max-log")
    ap.add_argument("--iterations", type=int, default=8)
    ap.add_argument("--ebn0", default="-2:10:1")
    ap.add_argument("--codewords", type=int, default=1_000_000, help="per Eb/N0 point, whole job")
    ap.add_argument("--batch", type=int, default=262144)
    ap.add_argument("--seed", type=int, default=2025)
    ap.add_argument("--interleaver", default="reference")
    ap.add_argument("--out", default=None)
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL) on the node; gloo to rehearse")
    ap.add_argument("--all-on-device0", action="store_true", help="every rank on GPU 0 (rehearsal on a 1-GPU box)")
    ap.add_argument("--dist-timeout", type=float, default=300.0, help="torch.distributed timeout (s)")
    a = ap.parse_args(argv)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.all_on_device0 and world > 1 and a.dist_backend == "nccl":
        ap.error("--all-on-device0 puts several ranks on one GPU, which RCCL cannot do: add --dist-backend gloo")
    # the codec touches no GPU until its first call: its inv_perm keys the sweep
    host_codec = M.DVBRCS2_Turbo(a.n, a.rate, a.iterations, algo=a.algo, interleaver=a.interleaver)
    cfg = sweep_config(a, host_codec.inv_perm)
    try:
        done = load_resume(a.out, cfg)
    except ValueError as e:
        ap.error(str(e))
    dev_idx = 0 if a.all_on_device0 else local
    torch.cuda.set_device(dev_idx)
    if world > 1:
        import datetime
        to = datetime.timedelta(seconds=a.dist_timeout)
        if a.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_idx), timeout=to)
        else:
            dist.init_process_group(a.dist_backend, timeout=to)
    device = torch.device("cuda", dev_idx)
    codec = M.DVBRCS2_Turbo(a.n, a.rate, a.iterations, algo=a.algo, interleaver=a.interleaver,
                            device=device.index)
    if world > 1:   # every rank must decode with the same de-interleaver
        S.check_same_interleaver(codec.inv_perm, dist, device if a.dist_backend == "nccl" else "cpu")
    pipe = DevicePipeline(codec, a.mod, a.batch, device)
    results = list(done.values())
    # one untimed batch first: code-object loading and first-launch costs stay out of
    # the first point's figures
    run_point(pipe, codec, a.mod, 2.0, 0, min(a.batch, 65536), a.batch, a.seed, device)
    for e in parse_points(a.ebn0):
        if e in done:
            continue
        start, count = S.shard_range(a.codewords, world, rank)
        t0 = time.time()
        times = []
        cnt = run_point(pipe, codec, a.mod, e, start, count, a.batch, ebn0_seed(a.seed, e), device, times)
        if world > 1 and a.dist_backend != "nccl":
            cnt = cnt.cpu()
        S.reduce_counters(cnt, dist if world > 1 else None)
        torch.cuda.synchronize()
        be, fe, ncw = (int(x) for x in cnt.tolist())
        dt = time.time() - t0
        rec = {"ebn0_db": e, "mod": a.mod, "n_couples": a.n, "rate": a.rate, "algo": a.algo,
               "interleaver": a.interleaver, "codewords": ncw,
               "bit_errors": be, "frame_errors": fe, "ber": be / (ncw * codec.k_info), "fer": fe / ncw,
               "seconds": dt, "codewords_per_s": ncw / dt, "gpus": world,
               # this rank's demap + decode (the bench's step) and decode alone, HIP events
               "step_ms": sum(t[0] for t in times), "decode_ms": sum(t[1] for t in times),
               "step_codewords_per_s": count / max(1e-9, sum(t[0] for t in times) * 1e-3),
               "decode_codewords_per_s": count / max(1e-9, sum(t[1] for t in times) * 1e-3)}
        results.append(rec)
        if rank == 0:
            print(json.dumps(rec), flush=True)
            if a.out:
                save_results(a.out, cfg, results)
    if world > 1:
        dist.destroy_process_group()
    return results


if __name__ == "__main__":
    main()
