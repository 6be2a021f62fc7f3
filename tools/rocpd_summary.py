"""Summarise rocprofv3 rocpd databases (kernel trace and PMC passes) into text/JSON under
profiles/.  Usage:
  python tools/rocpd_summary.py TAG gpurun_out/TAG   -> profiles/TAG_kernel_stats.txt,
                                                         profiles/TAG_pmc.txt,
                                                         profiles/hbm_traffic.json
Kernel durations are from the 'kernels' view (ns).  HBM traffic per launch follows
MI355X_MICROARCH.md "HBM [CDNA4]": FETCH_SIZE and WRITE_SIZE come from separate passes
(TCC slot limits); FETCH_SIZE is doubled (gfx950 tallies 128-B read requests at 64 B),
WRITE_SIZE is taken as is.  Both counters are in KiB.
"""
import glob
import json
import os
import sqlite3
import sys


def short(name):
    return name.split("(")[0].replace("void ", "")


def kernel_rows(db):
    rows = {}
    for name, dur in db.execute("select name, duration from kernels"):
        rows.setdefault(short(name), []).append(dur)
    return rows


def pmc_rows(db):
    out = {}
    for name, cname, val in db.execute("select name, counter_name, counter_value from pmc_events"):
        out.setdefault((short(name), cname), []).append(val)
    return out


def main():
    tag, d = sys.argv[1], sys.argv[2]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prof = os.path.join(root, "profiles")
    os.makedirs(prof, exist_ok=True)
    tr = glob.glob(os.path.join(d, "trace", "*.db"))
    lines = []
    if tr:
        rows = kernel_rows(sqlite3.connect(tr[0]))
        tot = sum(sum(v) for v in rows.values())
        lines.append("# rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 2 --warmup 1 --no-cpu  (%s)" % tag)
        lines.append("%-28s %7s %12s %12s %12s %12s %7s" % ("kernel", "calls", "total_ms", "avg_ms", "min_ms", "max_ms", "pct"))
        for k, v in sorted(rows.items(), key=lambda kv: -sum(kv[1])):
            lines.append("%-28s %7d %12.3f %12.3f %12.3f %12.3f %7.2f" % (
                k, len(v), sum(v) / 1e6, sum(v) / len(v) / 1e6, min(v) / 1e6, max(v) / 1e6, 100.0 * sum(v) / tot))
        open(os.path.join(prof, "%s_kernel_stats.txt" % tag), "w").write("\n".join(lines) + "\n")
        print("\n".join(lines))
    pm = {}
    for sub in ("pmc_fetch", "pmc_write"):
        f = glob.glob(os.path.join(d, sub, "*.db"))
        if f:
            pm.update(pmc_rows(sqlite3.connect(f[0])))
    if pm:
        pl = ["# rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) -- python3 bench.py --steps 1 --warmup 0 --no-cpu  (%s)" % tag,
              "%-28s %-11s %7s %16s" % ("kernel", "counter", "calls", "avg_KiB/launch")]
        for (k, c), v in sorted(pm.items()):
            pl.append("%-28s %-11s %7d %16.1f" % (k, c, len(v), sum(v) / len(v)))
        open(os.path.join(prof, "%s_pmc.txt" % tag), "w").write("\n".join(pl) + "\n")
        print("\n".join(pl))
        out = {"source": "%s: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py --steps 1 --warmup 0; "
                          "FETCH_SIZE x2 (gfx950 correction, MI355X_MICROARCH.md) + WRITE_SIZE" % tag}
        # timing names of pbrtgpu_last_timing <- device kernel names (the uninstrumented
        # template instances a bench frame runs)
        names = {"k_trace_closest": ("k_trace_pt<false, false>", "k_trace_closest<false, false>"),
                 "k_trace_shadow": ("k_trace_pt<true, false>", "k_trace_shadow<false, false>"),
                 "k_shade": tuple(sorted({kk for kk, _ in pm if kk.split("<")[0].endswith("k_shade")}))}
        for k, srcs in names.items():
            fetch = [x for s in srcs for x in pm.get((s, "FETCH_SIZE"), [])]
            write = [x for s in srcs for x in pm.get((s, "WRITE_SIZE"), [])]
            if not fetch or not write:
                continue
            # one frame was rendered per pass: total over its launches / launches
            fb = sum(fetch) * 1024.0
            wb = sum(write) * 1024.0
            n = len(fetch)
            out[k] = {"res": 700, "spp": 256, "launches": n, "fetch_bytes_raw_per_launch": fb / n,
                                    "write_bytes_per_launch": wb / len(write),
                                    "hbm_bytes_per_launch": (2.0 * fb + wb) / n}
        json.dump(out, open(os.path.join(prof, "hbm_traffic.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
