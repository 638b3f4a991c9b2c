"""Coded-BER Monte-Carlo sweep on MI355X (BASELINE.json configs[3]/[4]):
Eb/N0 points x codewords, sharded over GPUs with torchrun, resumable.

  python -m modulations_amd.ber --mod 256QAM --n 752 --rate 1/3 --ebn0=-2:10:1 \
      --codewords 10000000 --out ber_256qam.json
  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m modulations_amd.ber ...

Each rank owns a contiguous codeword range per point (sharding.shard_range),
generates it on its own device from a per-(rank, point) seed, runs the fused
demap + decode, and counts bit / frame errors; only those int64 counters are
all-reduced.  Finished points are written to --out after every point, and a
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


def run_point(pipe, codec, mod, ebn0, count, batch, seed, device):
    import torch
    from . import sharding as S
    cnt = torch.zeros(3, dtype=torch.int64, device=device)
    for i, (off, n) in enumerate(S.batches(count, batch)):
        info, syms, n0 = _gen(codec, n, mod, ebn0, seed + i, device)
        bits = pipe.run(syms, n0)[:n]
        e = (bits.to(torch.uint8) != info).sum(dim=1)
        cnt += torch.stack([e.sum(), (e > 0).sum(), torch.tensor(n, device=device)]).to(torch.int64)
    return cnt


def _gen(codec, n, mod, ebn0, seed, device):
    from .workload import make_symbols
    return make_symbols(codec, n, mod, ebn0, seed, device)


def main(argv=None):
    import torch
    import torch.distributed as dist
    from . import dvb_rcs2_turbo as M
    from . import sharding as S
    from .workload import DevicePipeline

    ap = argparse.ArgumentParser()
    ap.add_argument("--mod", default="256QAM")
    ap.add_argument("--n", type=int, default=752)
    ap.add_argument("--rate", default="1/3")
    ap.add_argument("--algo", default="max-log")
    ap.add_argument("--iterations", type=int, default=8)
    ap.add_argument("--ebn0", default="-2:10:1")
    ap.add_argument("--codewords", type=int, default=1_000_000, help="per Eb/N0 point, whole job")
    ap.add_argument("--batch", type=int, default=262144)
    ap.add_argument("--seed", type=int, default=2025)
    ap.add_argument("--interleaver", default="reference")
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", torch.cuda.current_device())
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
        cnt = run_point(pipe, codec, a.mod, e, count, a.batch, S.shard_seed(a.seed, rank, pi), device)
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
