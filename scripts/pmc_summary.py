"""Diagnostic: mean per-dispatch counter values of the step kernel from a
rocprofv3 --pmc output tree (default gpurun_out/pmcg)."""
import collections, csv, glob, sys
root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmcg"
needle = sys.argv[2] if len(sys.argv) > 2 else "step_kernel"
res = {}
for f in sorted(glob.glob(root + "/**/*counter_collection.csv", recursive=True)):
    by = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if needle in r["Kernel_Name"]:
            by[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    ids = sorted(by, key=int)[-5:]
    for c in (by[ids[0]] if ids else {}):
        res[c] = sum(by[i][c] for i in ids) / len(ids)
for c, v in sorted(res.items()):
    print(f"{c:36s} {v:18.1f}")
