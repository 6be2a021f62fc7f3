"""Device timeline of a rocprofv3 --kernel-trace run: where a render call's wall time goes.

Splits the trace into calls at host gaps longer than --split ms (the render calls of
tools/slice_run.py are separated by the host gather and the next call's setup), and per call
reports its span, the union of kernel-busy time, the idle time in gaps (and the gaps above
50 us: read-backs and host-side waits), and each kernel family's busy time (its own span,
overlapping kernels counted in each).

usage: python tools/timeline.py gpurun_out/TAG/trace [--split 3]
"""
import glob
import sqlite3
import sys

FAMILY = (("k_trace", "trace"), ("k_shade", "shade"), ("k_dl_", "shade"), ("k_regen", "shade"), ("k_accum", "accum"),
          ("k_mt_init", "mt_init"), ("k_live_list", "live_list"), ("k_spill", "spill"), ("k_apply", "spill"))


def family(name):
    n = name.split("(")[0].replace("void ", "").replace("pgd::", "")
    for pre, f in FAMILY:
        if n.startswith(pre):
            return f
    return "other:" + n[:24]


def rows(d):
    out = []
    for f in glob.glob(d + "/**/*.db", recursive=True):
        db = sqlite3.connect(f)
        cur = db.execute("select * from kernels limit 1")
        cols = [c[0] for c in cur.description]
        s = next(c for c in cols if c.lower() in ("start", "start_ns", "begin", "begin_ns"))
        e = next(c for c in cols if c.lower() in ("end", "end_ns"))
        out += [(a, b, n) for a, b, n in db.execute("select %s, %s, name from kernels" % (s, e))]
    return sorted(out)


def main():
    d = sys.argv[1]
    split = float(sys.argv[sys.argv.index("--split") + 1]) if "--split" in sys.argv else 3.0
    ks = rows(d)
    calls, cur = [], [ks[0]]
    for k in ks[1:]:
        if k[0] - max(x[1] for x in cur[-64:]) > split * 1e6:
            calls.append(cur)
            cur = []
        cur.append(k)
    calls.append(cur)
    for i, c in enumerate(calls):
        t0, t1 = c[0][0], max(x[1] for x in c)
        busy, gaps, big, end = 0, 0, [], t0
        fam = {}
        for a, b, n in c:
            fam[family(n)] = fam.get(family(n), 0) + (b - a)
            if a > end:
                gaps += a - end
                if a - end > 50e3:
                    big.append((a - end) / 1e3)
            busy += max(0, b - max(a, end))
            end = max(end, b)
        print("call %d: %d kernels, span %.2f ms, busy %.2f ms, idle %.2f ms (%d gaps > 50 us: %s)" % (
            i, len(c), (t1 - t0) / 1e6, busy / 1e6, gaps / 1e6, len(big), ", ".join("%.0f" % g for g in big[:24])))
        print("   per family (ms, own spans): " + ", ".join("%s %.2f" % (k, v / 1e6) for k, v in sorted(fam.items())))


if __name__ == "__main__":
    main()
