"""Summarise rocprofv3 rocpd databases (kernel traces and PMC passes of tools/gpu_profile.sh)
into profiles/.  Usage:
  python tools/rocpd_summary.py TAG gpurun_out/TAG CONFIG [OUTDIR (default profiles/)]
    -> profiles/TAG_kernel_stats.txt   per-kernel calls / total / avg / min / max (ns -> ms) of
                                       the default-mode trace and of the serial-mode trace
       profiles/TAG_pmc.txt            per-kernel PMC sums (FETCH, WRITE, SQ groups)
       profiles/hbm_traffic.json       configs[CONFIG][timing name]: HBM bytes per launch
Kernel durations are from the 'kernels' view (ns).  HBM traffic per launch follows
MI355X_MICROARCH.md "HBM [CDNA4]": FETCH_SIZE and WRITE_SIZE come from separate passes
(TCC slot limits); FETCH_SIZE is doubled (gfx950 tallies 128-B read requests at 64 B),
WRITE_SIZE is taken as is.  Both counters are in KiB.  The PMC passes render one serial-mode
frame, so each launch is counted once and alone on the device.
"""
import glob
import json
import os
import sqlite3
import sys

# timing names of pbrtgpu_last_timing <- device kernel name prefixes (uninstrumented instances)
NAMES = {"k_trace_closest": ("k_trace_pt<false, false>", "k_trace_closest<false, true>", "k_trace_inst<false, false>",
                             "k_trace_c4<false>"),
         "k_trace_shadow": ("k_trace_pt<true, false>", "k_trace_shadow<false, true>", "k_trace_inst<true, false>",
                            "k_trace_s4<false>", "k_trace_s4q<false>"),
         "k_shade": ("k_shade<", "k_dl_nee<", "k_dl_spec<", "k_regen<"),
         "k_accum": ("k_accum<",)}


def short(name):
    n = name.split("(")[0].replace("void ", "")
    return n[5:] if n.startswith("pgd::") else n


def timing_name(k):
    for t, pre in NAMES.items():
        if any(k.startswith(p) for p in pre):
            return t
    return None


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


def stats_lines(rows, title):
    tot = sum(sum(v) for v in rows.values())
    out = ["# " + title, "%-34s %7s %12s %12s %12s %12s %7s" % ("kernel", "calls", "total_ms", "avg_ms", "min_ms", "max_ms", "pct")]
    for k, v in sorted(rows.items(), key=lambda kv: -sum(kv[1])):
        out.append("%-34s %7d %12.3f %12.4f %12.4f %12.4f %7.2f" % (
            k[:34], len(v), sum(v) / 1e6, sum(v) / len(v) / 1e6, min(v) / 1e6, max(v) / 1e6, 100.0 * sum(v) / tot))
    return out


def main():
    tag, d, cfg = sys.argv[1], sys.argv[2], sys.argv[3]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prof = os.path.join(root, "profiles")
    out = sys.argv[4] if len(sys.argv) > 4 else prof   # the GPU box: a directory under gpurun_out
    os.makedirs(out, exist_ok=True)
    lines = []
    for sub, title in (("trace", "rocprofv3 --kernel-trace --stats -- python3 bench.py --config %s --no-cpu --no-roofline "
                                 "--steps 2 --warmup 1   (default mode: two lanes + shadow stream, spans overlap)"),
                       ("trace_serial", "rocprofv3 --kernel-trace --stats -- python3 bench.py --config %s --no-cpu "
                                        "--no-roofline --steps 1 --warmup 1 --serial   (exclusive kernel durations)")):
        f = glob.glob(os.path.join(d, sub, "**", "*.db"), recursive=True)
        if f:
            lines += stats_lines(kernel_rows(sqlite3.connect(f[0])), (title % cfg) + "  [%s]" % tag) + [""]
    if lines:
        open(os.path.join(out, "%s_kernel_stats.txt" % tag), "w").write("\n".join(lines))
        print("\n".join(lines))
    pm = {}
    for sub in ("pmc_fetch", "pmc_write", "pmc_sq1", "pmc_sq2", "pmc_lds", "pmc_tcc"):
        for f in glob.glob(os.path.join(d, sub, "**", "*.db"), recursive=True):
            for kk, v in pmc_rows(sqlite3.connect(f)).items():
                pm.setdefault(kk, []).extend(v)
    if not pm:
        return
    pl = ["# rocprofv3 --pmc <group> (separate passes) -- python3 bench.py --config %s --steps 1 --warmup 0 --serial "
          "--no-cpu --no-roofline  [%s]" % (cfg, tag),
          "%-34s %-22s %7s %18s %18s" % ("kernel", "counter", "calls", "sum", "avg/launch")]
    per = {}
    for (k, c), v in sorted(pm.items()):
        if k.startswith("__amd"):
            continue
        pl.append("%-34s %-22s %7d %18.1f %18.1f" % (k[:34], c, len(v), sum(v), sum(v) / len(v)))
        t = timing_name(k)
        if t:
            e = per.setdefault(t, {})
            e.setdefault(c, [0.0, 0])
            e[c][0] += sum(v)
            e[c][1] += len(v)
    for t, cs in sorted(per.items()):
        if "SQ_WAVE_CYCLES" in cs:
            wc = cs["SQ_WAVE_CYCLES"][0]
            parts = ["%s %.1f%%" % (c, 100.0 * cs[c][0] / wc) for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")
                     if c in cs]
            pl.append("# %s: %s of SQ_WAVE_CYCLES" % (t, ", ".join(parts)))
        if "TCC_HIT_sum" in cs and "TCC_MISS_sum" in cs:
            h, m = cs["TCC_HIT_sum"][0], cs["TCC_MISS_sum"][0]
            pl.append("# %s: TCC (L2) hit rate %.1f%% (%d hits, %d misses)" % (t, 100.0 * h / max(h + m, 1), h, m))
        if "SQ_INSTS_VALU" in cs and "SQ_WAVES" in cs:
            pl.append("# %s: VALU insts / wave %.0f, VMEM_RD / wave %.1f, VMEM_WR / wave %.1f" % (
                t, cs["SQ_INSTS_VALU"][0] / cs["SQ_WAVES"][0], cs.get("SQ_INSTS_VMEM_RD", [0])[0] / cs["SQ_WAVES"][0],
                cs.get("SQ_INSTS_VMEM_WR", [0])[0] / cs["SQ_WAVES"][0]))
    open(os.path.join(out, "%s_pmc.txt" % tag), "w").write("\n".join(pl) + "\n")
    print("\n".join(pl))
    tf = os.path.join(prof, "hbm_traffic.json")
    tr = json.load(open(tf)) if os.path.exists(tf) else {}
    tf = os.path.join(out, "hbm_traffic.json")
    if os.path.exists(tf):   # an earlier config of the same run
        tr = json.load(open(tf))
    if "configs" not in tr:
        tr = {"configs": {}}
    ent = {"source": "%s: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (separate) of bench.py --config %s --steps 1 "
                     "--warmup 0 --serial; FETCH_SIZE x2 (gfx950 correction, MI355X_MICROARCH.md) + WRITE_SIZE" % (tag, cfg)}
    # per launch of the family's first kernel: bench.py times a DirectLighting shade step (k_shade,
    # k_dl_nee, k_dl_spec, k_regen) as one k_shade launch, so its bytes are the step's
    lead = {}
    for (k, c), v in pm.items():
        t = timing_name(k)
        if t and c == "FETCH_SIZE" and k.startswith(NAMES[t][0]):
            lead[t] = lead.get(t, 0) + len(v)
    for t, cs in per.items():
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            fb, n = cs["FETCH_SIZE"][0] * 1024.0, lead.get(t) or cs["FETCH_SIZE"][1]
            wb, nw = cs["WRITE_SIZE"][0] * 1024.0, lead.get(t) or cs["WRITE_SIZE"][1]
            ent[t] = {"launches": n, "fetch_bytes_raw_per_launch": fb / n, "write_bytes_per_launch": wb / nw,
                      "hbm_bytes_per_launch": 2.0 * fb / n + wb / nw}
    tr["configs"][cfg] = ent
    json.dump(tr, open(tf, "w"), indent=1)


if __name__ == "__main__":
    main()
