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
only those int64 counters are all-reduced.  Finished points are written to --out after every point, and a
rerun skips them (checkpoint / resume).
"""
from __future__ import annotations

import argparse
import json
import os
import time

import numpy as np


def parse_points(spec):
    if ":" in spec:
        a, b, s = (float(x) for x in spec.split(":"))
        return [round(a + i * s, 6) for i in range(int(round((b - a) / s)) + 1)]
    return [float(x) for x in spec.split(",")]


def run_point(pipe, codec, mod, ebn0, start, count, batch, seed, device):
    """Bit errors, frame errors and codewords of global codewords
    [start, start + count) at one Eb/N0 point.  The data of codeword g is a
    counter-based stream of (seed, g) (workload.make_symbols), so the counters
    do not depend on the batch size or on how the job is sharded."""
    import torch
    from . import sharding as S
    from .workload import count_errors, make_symbols
    cnt = torch.zeros(3, dtype=torch.int64, device=device)
    for off, n in S.batches(count, batch):
        _, syms, n0 = make_symbols(codec, n, mod, ebn0, seed, device, cw0=start + off, want_info=False)
        bits = pipe.run(syms, n0)[:n]
        e = count_errors(codec, bits, seed, cw0=start + off)
        cnt += torch.stack([e.sum(dtype=torch.int64), (e > 0).sum(), torch.tensor(n, device=device)]).to(torch.int64)
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
    a = ap.parse_args(argv)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev_idx = 0 if a.all_on_device0 else local
    torch.cuda.set_device(dev_idx)
    if world > 1:
        if a.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_idx))
        else:
            dist.init_process_group(a.dist_backend)
    device = torch.device("cuda", dev_idx)
    codec = M.DVBRCS2_Turbo(a.n, a.rate, a.iterations, algo=a.algo, interleaver=a.interleaver,
                            device=device.index)
    pipe = DevicePipeline(codec, a.mod, a.batch, device)
    done = {}
    if a.out and os.path.exists(a.out):
        done = {float(r["ebn0_db"]): r for r in json.load(open(a.out))}
    results = list(done.values())
    for pi, e in enumerate(parse_points(a.ebn0)):
        if e in done:
            continue
        start, count = S.shard_range(a.codewords, world, rank)
        t0 = time.time()
        cnt = run_point(pipe, codec, a.mod, e, start, count, a.batch, S.point_seed(a.seed, pi), device)
        if world > 1 and a.dist_backend != "nccl":
            cnt = cnt.cpu()
        S.reduce_counters(cnt, dist if world > 1 else None)
        torch.cuda.synchronize()
        be, fe, ncw = (int(x) for x in cnt.tolist())
        rec = {"ebn0_db": e, "mod": a.mod, "n_couples": a.n, "rate": a.rate, "algo": a.algo, "codewords": ncw,
               "bit_errors": be, "frame_errors": fe, "ber": be / (ncw * codec.k_info), "fer": fe / ncw,
               "seconds": time.time() - t0, "gpus": world}
        results.append(rec)
        if rank == 0:
            print(json.dumps(rec), flush=True)
            if a.out:
                json.dump(sorted(results, key=lambda r: r["ebn0_db"]), open(a.out, "w"), indent=1)
    if world > 1:
        dist.destroy_process_group()
    return results


if __name__ == "__main__":
    main()
