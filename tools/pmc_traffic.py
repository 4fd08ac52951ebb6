"""Parse the two rocprofv3 --pmc passes of tools/pmc_traffic.sh into per-launch HBM bytes per stage.

gfx950 correction (MI355X_MICROARCH.md 'HBM'; cdna_hip_programming.md section 7): FETCH_SIZE and WRITE_SIZE
are in KiB; FETCH_SIZE reports exactly half the bytes of a wide coalesced streaming read, so
    traffic = (2 * FETCH_SIZE + WRITE_SIZE) * 1024
The raw counters are kept next to the corrected figure (other access widths are uncalibrated).

The third pass (FP64) holds the FP64 VALU counters: SQ_INSTS_VALU_FLOPS_FP64 (+ _TRANS) is the FP64 FLOP count of
the launch (per active lane, FMA = 2), SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F64 the FP64 wave-instructions issued; bench.py
reads both for the pose LM's FP64 roofline."""
import csv
import glob
import json
import os
import sys

STAGE_OF = {"detect_kernel": "detect", "topk_kernel": "topk", "brief_kernel": "brief",
            "match_finalize_kernel": "finalize", "match_kernel": "match", "match_fp4_kernel": "match",
            "track_build_kernel": "track_edges",
            "pose_lm_kernel": "track_pose"}


def stage(kernel_name):
    # kernel names as rocprofv3 prints them: "yavo::match_kernel(...)", "void yavo::detect_kernel<true>(...)",
    # "yavo::geom::pose_lm_kernel(...)"
    base = kernel_name.split("(")[0].split("<")[0].split("::")[-1].strip()
    return STAGE_OF.get(base)


def load(out_dir, counter, pass_dir=None):
    files = glob.glob(os.path.join(out_dir, f"pmc_{pass_dir or counter}", "**", "*counter_collection*.csv"),
                      recursive=True)
    per = {}
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name") or row.get("Kernel-Name") or ""
                if (row.get("Counter_Name") or "") != counter:
                    continue
                st = stage(name)
                if st is None:
                    continue
                per.setdefault(st, []).append(float(row.get("Counter_Value") or 0.0))
    return per


def main():
    out_dir = sys.argv[1]
    frames = 2048  # bench.py's default (--frames)
    args = sys.argv[2:]
    if "--frames" in args:
        frames = int(args[args.index("--frames") + 1])
    fetch = load(out_dir, "FETCH_SIZE")
    write = load(out_dir, "WRITE_SIZE")
    res = {"frames_per_step": frames, "units": "bytes per launch", "per_launch_bytes": {}, "raw_kib": {},
           "formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE half-count correction)"}
    for st in sorted(set(fetch) | set(write)):
        f = fetch.get(st, [])
        w = write.get(st, [])
        # skip the warm-up launch: use the last three dispatches of each stage
        f = f[-3:] if len(f) > 3 else f
        w = w[-3:] if len(w) > 3 else w
        fm = sum(f) / len(f) if f else 0.0
        wm = sum(w) / len(w) if w else 0.0
        res["raw_kib"][st] = {"FETCH_SIZE": fm, "WRITE_SIZE": wm, "dispatches": [len(f), len(w)]}
        res["per_launch_bytes"][st] = int((2 * fm + wm) * 1024)
    fp64 = {c: load(out_dir, c, "FP64") for c in ("SQ_INSTS_VALU_FLOPS_FP64", "SQ_INSTS_VALU_FLOPS_FP64_TRANS",
                                                   "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64",
                                                   "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64")}
    stages = sorted(set().union(*[set(v) for v in fp64.values()]))
    if stages:
        res["fp64_per_launch"] = {}
        for st in stages:
            vals = {}
            for c, per in fp64.items():
                x = per.get(st, [])
                x = x[-3:] if len(x) > 3 else x
                vals[c] = sum(x) / len(x) if x else 0.0
            if not any(vals.values()):
                continue
            res["fp64_per_launch"][st] = {
                "flops": vals["SQ_INSTS_VALU_FLOPS_FP64"] + vals["SQ_INSTS_VALU_FLOPS_FP64_TRANS"],
                "wave_instructions": sum(vals[c] for c in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64",
                                                           "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64")),
                "raw": vals}
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    # the code the counters were taken on: bench.py uses `traffic` only while its kernel sources hash the same
    sys.path.insert(0, root)
    import bench
    res["source_sha256"] = bench.kernel_source_digest()
    res["commit"] = os.environ.get("YAVO_COMMIT", "")
    path = os.path.join(root, "profiles", "pmc_traffic.json")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    json.dump(res, open(path, "w"), indent=1)
    json.dump(res, open(os.path.join(out_dir, "pmc_traffic.json"), "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
