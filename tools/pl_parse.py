import collections, csv, sys
def load(path):
    rows = list(csv.DictReader(open(path)))
    d = collections.OrderedDict()
    for r in rows:
        if "k_turbo_decode" not in r["Kernel_Name"]: continue
        k = int(r["Dispatch_Id"])
        e = d.setdefault(k, {"ms": (float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) / 1e6})
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0) + float(r["Counter_Value"])
    return list(d.values())
for name in sys.argv[1:]:
    print("==", name)
    for e in load(name):
        extra = ""
        if "TCC_EA0_RDREQ_LEVEL_sum" in e:
            extra = f"  avg_rd_inflight/req={e['TCC_EA0_RDREQ_LEVEL_sum']/e['TCC_EA0_RDREQ_sum']:.1f}"
        if "TCP_UTCL1_TRANSLATION_MISS_sum" in e:
            extra = f"  miss_rate={e['TCP_UTCL1_TRANSLATION_MISS_sum']/e['TCP_UTCL1_REQUEST_sum']:.4f}"
        print(f"{e['ms']:7.2f} ms " + " ".join(f"{k.replace('TCP_','').replace('TCC_','').replace('_sum','')}={v:.3e}" for k, v in e.items() if k != "ms") + extra)
