#!/usr/bin/env python3
"""Summarise a rocprofv3 run directory (kernel trace + PMC passes) of bench.py
into profiles/<round>_summary.{json,md}.

HBM traffic per launch follows MI355X_MICROARCH.md §HBM: FETCH_SIZE and
WRITE_SIZE come from separate --pmc passes, are in KiB, and on gfx950 FETCH_SIZE
reads exactly half the bytes of a wide coalesced streaming read, so
hbm_bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024.

usage: tools/prof_summary.py gpurun_out/r01 profiles/r01 [batch] [workload string: stamp profiles/traffic.json]
"""
import collections
import csv
import json
import os
import sys


def short(name):
    for k in ("k_turbo_decode_syms", "k_turbo_decode_logmap", "k_turbo_decode", "k_demap_planes", "k_workload",
              "k_count_errors", "k_siso_spl", "k_depuncture", "k_encode", "k_siso_batch", "k_demap_fix",
              "k_demap", "k_map", "k_demod", "k_fir_up", "k_fir_dec", "k_fir", "k_absmax", "k_quantize",
              "k_dequantize"):
        if k in name:
            return k
    return name[:60]


def full_size(rows, dur):
    """Drop dispatches shorter than 30 % of the kernel's longest: the
    decoder's one-iteration workspace placement probes (tdec_reserve) run the
    same kernel and would otherwise dilute the per-launch averages."""
    by = collections.defaultdict(list)
    for r in rows:
        by[short(r["Kernel_Name"])].append(r)
    keep = []
    for k, rs in by.items():
        longest = max(dur(r) for r in rs)
        keep += [r for r in rs if dur(r) >= 0.3 * longest]
    return keep


def span(r):
    return float(r["End_Timestamp"]) - float(r["Start_Timestamp"])


def pmc(path):
    agg = collections.defaultdict(list)
    for r in full_size(list(csv.DictReader(open(path))), span):
        agg[(short(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FETCH_FACTOR = 2.0   # MI355X_MICROARCH.md: FETCH_SIZE counts half of a wide streaming read (re-checked: r02_fetch_cal)


def main(src, dst, batch=1 << 20, workload=None):
    batch = int(batch)
    out = {"source": src, "batch_codewords": batch, "kernels": {}}
    trace = full_size(list(csv.DictReader(open(os.path.join(src, "kt", "kt_kernel_trace.csv")))), span)
    durs = collections.defaultdict(list)
    for r in trace:
        durs[short(r["Kernel_Name"])].append(span(r) / 1e6)
    for k, v in durs.items():
        if k.startswith("k_"):
            out["kernels"][k] = {"calls": len(v), "avg_ms": sum(v) / len(v), "min_ms": min(v), "max_ms": max(v)}
    counters = {}
    for sub in ("fetch/f", "write/w", "sq/s", "tcc/t"):
        p = os.path.join(src, sub + "_counter_collection.csv")
        if os.path.exists(p):
            counters.update(pmc(p))
    for k, d in out["kernels"].items():
        c = {cn: v for (kk, cn), v in counters.items() if kk == k}
        d["counters"] = c
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            rd = FETCH_FACTOR * c["FETCH_SIZE"] * 1024
            wr = c["WRITE_SIZE"] * 1024
            d["hbm_read_bytes"] = rd
            d["hbm_write_bytes"] = wr
            d["hbm_bytes_per_launch"] = rd + wr
            d["hbm_GBps"] = (rd + wr) / (d["avg_ms"] * 1e-3) / 1e9
            d["hbm_bytes_per_codeword"] = (rd + wr) / batch
        if "TCC_HIT_sum" in c:
            d["l2_hit_rate"] = c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
        if "SQ_WAVE_CYCLES" in c:
            d["wait_any_frac"] = c.get("SQ_WAIT_ANY", 0) / c["SQ_WAVE_CYCLES"]
            d["wait_inst_any_frac"] = c.get("SQ_WAIT_INST_ANY", 0) / c["SQ_WAVE_CYCLES"]
            d["active_inst_any_frac"] = c.get("SQ_ACTIVE_INST_ANY", 0) / c["SQ_WAVE_CYCLES"]
            d["valu_insts_per_codeword"] = c.get("SQ_INSTS_VALU", 0) * 64 / batch
            # clock from GRBM_GUI_ACTIVE (summed over the 8 XCDs)
            clk = 2.4e9
            if "GRBM_GUI_ACTIVE" in c:
                clk = c["GRBM_GUI_ACTIVE"] / 8 / (d["avg_ms"] * 1e-3)
                d["clock_GHz"] = clk / 1e9
            # VALU issue-busy share: wave-instructions x 2 cycles (SIMD-32) / (1024 SIMDs x cycles)
            d["valu_busy_est"] = c.get("SQ_INSTS_VALU", 0) * 2 / (1024 * clk * d["avg_ms"] * 1e-3)
    json.dump(out, open(dst + "_summary.json", "w"), indent=1)
    if workload:   # stamp profiles/traffic.json with the library this run loaded
        import hashlib
        lib = os.path.join(ROOT, "modulations_amd", "lib", "libtdec.so")
        sha = hashlib.sha256(open(lib, "rb").read()).hexdigest()
        sys.path.insert(0, ROOT)
        from modulations_amd.build import build_info
        src_sha = (build_info(lib) or {}).get("src_sha256")
        tf = os.path.join(ROOT, "profiles", "traffic.json")
        tr = json.load(open(tf)) if os.path.exists(tf) else {}
        for k in ("k_turbo_decode", "k_turbo_decode_logmap"):
            d = out["kernels"].get(k)
            if not d or "hbm_bytes_per_codeword" not in d:
                continue
            ent = tr.get(k, {})
            if not isinstance(ent, dict) or "workload" in ent:   # round-1 flat format
                ent = {}
            ent[workload] = {"hbm_bytes_per_codeword": d["hbm_bytes_per_codeword"],
                             "hbm_read_bytes_per_codeword": d["hbm_read_bytes"] / batch,
                             "hbm_write_bytes_per_codeword": d["hbm_write_bytes"] / batch,
                             "avg_ms": d["avg_ms"], "lib_sha256": sha, "src_sha256": src_sha, "source": dst + "_summary.json",
                             "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes (KiB); "
                                       f"FETCH_SIZE x {FETCH_FACTOR} (gfx950 read calibration, "
                                       "profiles/r02_fetch_cal.txt); per launch / codewords per launch"}
            tr[k] = ent
        json.dump(tr, open(tf, "w"), indent=1)
    with open(dst + "_summary.md", "w") as f:
        f.write(f"# rocprofv3 summary ({src}), batch = {batch} codewords\n\n")
        f.write("| kernel | calls | avg ms | HBM GB/launch | HBM GB/s | B/codeword | L2 hit | VALU busy (est) | wait_any | wait_inst | clock GHz |\n")
        f.write("|---|---|---|---|---|---|---|---|---|---|---|\n")
        for k, d in out["kernels"].items():
            f.write(f"| {k} | {d['calls']} | {d['avg_ms']:.2f} | {d.get('hbm_bytes_per_launch', 0) / 1e9:.1f} | "
                    f"{d.get('hbm_GBps', 0):.0f} | {d.get('hbm_bytes_per_codeword', 0):.0f} | "
                    f"{d.get('l2_hit_rate', 0):.2f} | {d.get('valu_busy_est', 0):.2f} | {d.get('wait_any_frac', 0):.2f} | "
                    f"{d.get('wait_inst_any_frac', 0):.2f} | {d.get('clock_GHz', 0):.2f} |\n")
    print(open(dst + "_summary.md").read())


if __name__ == "__main__":
    main(*sys.argv[1:])
