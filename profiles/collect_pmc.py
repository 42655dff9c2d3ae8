"""Collect HBM traffic of the step kernel with rocprofv3 PMC counters
(run on the GPU box from the repo root; spawns rocprofv3, never touches the
GPU itself).

Per MI355X_MICROARCH.md §HBM / cdna_hip_programming.md §7: FETCH_SIZE and
WRITE_SIZE in separate --pmc passes (TCC slots), values in KB; on gfx950
FETCH_SIZE reports half the bytes of a wide coalesced stream, other widths
are uncalibrated — so a calibration kernel with the step kernel's own state
access pattern (8 B per lane, SoA) is measured too, and both the
guide-corrected and the calibrated figures are written to
profiles/pmc_traffic.json, keyed "<config>_<dtype>".
"""
import csv, glob, json, os, subprocess, sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out", "pmc_traffic")
os.makedirs(OUT, exist_ok=True)
env = dict(os.environ, TMPDIR="/tmp")


def run_pmc(counter, cmd, tag):
    d = os.path.join(OUT, f"{tag}_{counter}")
    subprocess.run(["timeout", "-k", "10", "600", "rocprofv3", "--pmc", counter, "--output-format", "csv",
                    "-d", d, "-o", "run", "--"] + cmd, check=True, env=env, cwd=ROOT,
                   stdout=subprocess.DEVNULL)
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            vals.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    return vals


def mean_for(vals, needle):
    xs = [v for k, vs in vals.items() if needle in k for v in vs]
    return sum(xs) / len(xs) if xs else None


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
    dtype = sys.argv[2] if len(sys.argv) > 2 else "f64"
    P = int(sys.argv[3]) if len(sys.argv) > 3 else 1      # > 1: one rank's step kernel of a P-way strong split
    suffix = sys.argv[4] if len(sys.argv) > 4 else ""     # e.g. "_tile" (run with RBHIP_TILE=1): a key of its own
    # calibration: known-byte kernel with the state access pattern
    exe = "/tmp/calib_fetch"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-o", exe,
                    os.path.join(ROOT, "profiles", "calib_fetch.hip")], check=True)
    n = 1 << 24
    known = n * 8 * 13
    cf = mean_for(run_pmc("FETCH_SIZE", [exe, str(n)], "calib"), "soa_rw")
    cw = mean_for(run_pmc("WRITE_SIZE", [exe, str(n)], "calib"), "soa_rw")
    read_factor = known / (cf * 1024.0)
    write_factor = known / (cw * 1024.0)
    if P == 1:
        # bench.py's default window (steps 51-450 captured, 451-850 timed:
        # C4's pile-ups included)
        bench = [sys.executable, "bench.py", "--config", cfg, "--dtype", dtype, "--no-cpu-baseline"]
    else:
        # P shards stepped in one process (scripts/shard_step_run.py): each
        # rank's step kernel over its own slice, tables as in a P-GPU run
        bench = [sys.executable, "scripts/shard_step_run.py", "--config", cfg, "--dtype", dtype, "--P", str(P)]
    tag = (cfg if P == 1 else f"{cfg}_p{P}") + suffix
    # the hashed-cell keys average the hashed step kernels ("rb::step_kernel",
    # which "rb::tile_step_kernel" does not contain), "_tile" the tile kernel
    needle = "tile_step_kernel" if suffix == "_tile" else "rb::step_kernel"
    fv, wv = run_pmc("FETCH_SIZE", bench, tag), run_pmc("WRITE_SIZE", bench, tag)
    f = mean_for(fv, needle)
    w = mean_for(wv, needle)
    guide = f * 1024.0 * 2.0 + w * 1024.0
    calibrated = f * 1024.0 * read_factor + w * 1024.0 * write_factor
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    data = json.load(open(path)) if os.path.exists(path) else {}
    key = (f"{cfg}_{dtype}" if P == 1 else f"{cfg}_{dtype}_p{P}") + suffix
    import hashlib
    lib = os.path.join(ROOT, "rigidbody-simulation_amd", "rbhip", "librbhip.so")
    data[key] = {
        # the library build the counters saw (bench.py flags a line whose
        # library differs: the figures may then be stale)
        "librbhip_sha16": hashlib.sha256(open(lib, "rb").read()).hexdigest()[:16],
        "fetch_size_kb_per_launch": f, "write_size_kb_per_launch": w,
        "hbm_bytes_per_launch": guide,
        "hbm_bytes_per_launch_lower": f * 1024.0 + w * 1024.0,
        "hbm_bytes_per_launch_calibrated": calibrated,
        "correction": "guide: FETCH_SIZE*1024*2 + WRITE_SIZE*1024 (gfx950 half-count of wide reads); "
                      "calibrated: factors from profiles/calib_fetch.hip (8 B/lane SoA, known bytes)",
        "calibration": {"known_bytes": known, "fetch_kb": cf, "write_kb": cw,
                        "read_factor": read_factor, "write_factor": write_factor},
        "kernel": "step kernel", "per": "launch",
        "note": "FETCH_SIZE counts requests leaving L2, Infinity-Cache (MALL) hits included; the x2 "
                "read correction holds for 128-B streaming requests (the state arrays), random 64-B "
                "gathers (buckets, candidate snapshots) count once: the true figure lies between "
                "hbm_bytes_per_launch_lower and hbm_bytes_per_launch",
    }
    json.dump(data, open(path, "w"), indent=1)
    print(json.dumps(data[key], indent=1))


if __name__ == "__main__":
    main()
