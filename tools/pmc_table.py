"""Per-kernel sums of every PMC counter in rocpd databases under a directory.
Usage: python tools/pmc_table.py gpurun_out/TAG/p1 [more dirs]"""
import glob
import sqlite3
import sys


def short(name):
    return name.split("(")[0].replace("void ", "")


tot = {}
for d in sys.argv[1:]:
    for f in glob.glob(d + "/**/*.db", recursive=True):
        db = sqlite3.connect(f)
        for name, cname, val in db.execute("select name, counter_name, counter_value from pmc_events"):
            k = short(name)
            if k.startswith("__amd"):
                continue
            tot.setdefault(k, {}).setdefault(cname, 0.0)
            tot[k][cname] += val
for k, cs in sorted(tot.items()):
    print(k)
    wc = cs.get("SQ_WAVE_CYCLES")
    for c, v in sorted(cs.items()):
        extra = ""
        if wc and c.startswith(("SQ_WAIT", "SQ_ACTIVE")):
            extra = "  (%.1f%% of wave cycles)" % (100.0 * v / wc)
        print("   %-28s %16.0f%s" % (c, v, extra))
    if "SQ_INSTS_VALU" in cs and "SQ_WAVES" in cs:
        print("   VALU insts / wave %.0f, VMEM_RD / wave %.1f" % (cs["SQ_INSTS_VALU"] / cs["SQ_WAVES"],
                                                                cs.get("SQ_INSTS_VMEM_RD", 0) / cs["SQ_WAVES"]))
