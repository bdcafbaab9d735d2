"""Summarise tools/profile.sh output into profiles/ (tracked).

  python tools/prof_summary.py gpurun_out/prof_r05_flat profiles/r05_flat --kernel multi --f64 --traffic

Writes <dst>_kernel_stats.csv (rocprofv3 --stats, verbatim), <dst>_summary.json
(average step_kernel duration over the timed dispatches, PMC per launch) and,
with --traffic, updates profiles/traffic.json (read by bench.py for
roofline.traffic).  FETCH_SIZE is doubled per MI355X_MICROARCH.md (gfx950
reports half the bytes of wide coalesced reads); WRITE_SIZE is taken as is.
"""
import argparse
import csv
import json
import shutil
from pathlib import Path

KERNEL = "step_kernel"
SEL = {"which": "fast"}  # --kernel: fast (step_kernel<T,false>), pred (the route-0 predicted full kernel),
#                          multi (multi_step_kernel<T>, bb_step_multi) or pair (the relief pair: both
#                          relief_pair_kernel launches of one bb_step_multi call, summed)


def is_fast(name):
    """The fast step kernel step_kernel<T, false>."""
    return KERNEL in name and ", false>" in name


def is_full(name):
    return KERNEL in name and ", true>" in name


def select_ids(recs):
    """Dispatch ids of the selected kernel.  pred: on route 0 the predicted full kernel is
    the step_kernel<T,true> dispatch launched right before each fast dispatch (the
    hand-over full kernel comes after it)."""
    recs = sorted(recs, key=lambda r: int(r["Dispatch_Id"]))
    if SEL["which"] == "pair":
        one = [int(r["Dispatch_Id"]) for r in recs if "relief_pair1_kernel" in r["Kernel_Name"]]
        SEL["pair_one"] = bool(one)
        return one or [int(r["Dispatch_Id"]) for r in recs if "relief_pair_kernel" in r["Kernel_Name"]]
    if SEL["which"] == "multi":
        # multi_step_kernel<T, false> (the fast launch; the finish launch <T, true> only reads park[]
        # on flat), or the single inline launch <T, true> under BB_MULTI_PARK=0, or relief_multi_kernel
        # relief banks: relief_multi_kernel (with the adaptive route the gated multi-step launches
        # of a queue launch exit at once; a parked launch would show as multi_step_kernel<T, false>)
        rq = [int(r["Dispatch_Id"]) for r in recs if "relief_multi_kernel" in r["Kernel_Name"]]
        if rq:
            return rq
        ms = [r for r in recs if "multi_step_kernel" in r["Kernel_Name"]]
        if any(", false>" in r["Kernel_Name"] for r in ms):
            ms = [r for r in ms if ", false>" in r["Kernel_Name"]]
        return [int(r["Dispatch_Id"]) for r in ms]
    if SEL["which"] == "fast":
        return [int(r["Dispatch_Id"]) for r in recs if is_fast(r["Kernel_Name"])]
    out, last_full = [], None
    for r in recs:
        if is_full(r["Kernel_Name"]):
            last_full = int(r["Dispatch_Id"])
        elif is_fast(r["Kernel_Name"]) and last_full is not None:
            out.append(last_full)
            last_full = None
    return out


def rows(p):
    with open(p) as f:
        return list(csv.DictReader(f))


def counters(p, names, last):
    per = {}
    rr = rows(p)
    seen = {}
    for r in rr:
        seen.setdefault(int(r["Dispatch_Id"]), r)
    keep = set(select_ids(list(seen.values())))
    for r in rr:
        if int(r["Dispatch_Id"]) not in keep:
            continue
        d = per.setdefault(int(r["Dispatch_Id"]), {})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    ids = sorted(per)
    if SEL["which"] == "pair" and not SEL.get("pair_one"):  # one launch = its two relief_pair_kernel dispatches
        grp = [ids[i:i + 2] for i in range(0, len(ids) - 1, 2)][-last:]
        return {n: sum(sum(per[i].get(n, 0.0) for i in g) for g in grp) / len(grp) for n in names}, len(grp)
    ids = ids[-last:]
    return {n: sum(per[i].get(n, 0.0) for i in ids) / len(ids) for n in names}, len(ids)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("dst")
    ap.add_argument("--timed", type=int, default=1, help="timed dispatches at the end of the trace run (bench.py's "
                                                         "timed window is the last launch with --no-per-step)")
    ap.add_argument("--pmc-last", type=int, default=1)
    ap.add_argument("--traffic", action="store_true")
    ap.add_argument("--kernel", default="fast", choices=["fast", "pred", "multi", "pair"])
    ap.add_argument("--f64", action="store_true", help="also summarise the FP64 VALU instruction pass (sq64)")
    a = ap.parse_args()
    SEL["which"] = a.kernel
    src, dst = Path(a.src), Path(a.dst)
    dst.parent.mkdir(parents=True, exist_ok=True)
    shutil.copy(src / "trace" / "run_kernel_stats.csv", str(dst) + "_kernel_stats.csv")
    allr = rows(src / "trace" / "run_kernel_trace.csv")
    keep = set(select_ids(allr))
    tr = [r for r in allr if int(r["Dispatch_Id"]) in keep]
    tr.sort(key=lambda r: int(r["Start_Timestamp"]))
    if a.kernel == "pair" and not SEL.get("pair_one"):  # a launch: first start to last end of its two dispatches
        tr.sort(key=lambda r: int(r["Dispatch_Id"]))
        grp = [tr[i:i + 2] for i in range(0, len(tr) - 1, 2)][-a.timed:]
        timed = [g[0] for g in grp]
        durs = [(max(int(r["End_Timestamp"]) for r in g) - min(int(r["Start_Timestamp"]) for r in g)) * 1e-6
                for g in grp]
    else:
        timed = tr[-a.timed:]
        durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6 for r in timed]
    bench = json.loads((src / "bench_trace.json").read_text())
    out = {
        "kernel": timed[0]["Kernel_Name"],
        "timed_dispatches": len(timed),
        "avg_ms_rocprof": sum(durs) / len(durs),
        "min_ms": min(durs), "max_ms": max(durs),
        "bench_kernel_ms_hip_events": bench["roofline"]["kernel_ms"],
        "bench_kernel_ms_all": bench["roofline"].get("kernel_ms_all"),
        "bench_value": bench["value"],
        "bench_config": bench["config"],
        "vgpr": timed[0].get("VGPR_Count"), "agpr": timed[0].get("Accum_VGPR_Count"),
        "sgpr": timed[0].get("SGPR_Count"), "lds": timed[0].get("LDS_Block_Size"),
        "scratch": timed[0].get("Scratch_Size"),
    }
    f, nf = counters(src / "fetch" / "run_counter_collection.csv", ["FETCH_SIZE", "GRBM_GUI_ACTIVE"], a.pmc_last)
    w, nw = counters(src / "write" / "run_counter_collection.csv", ["WRITE_SIZE"], a.pmc_last)
    sqn = ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
           "SQ_ACTIVE_INST_ANY", "SQ_WAVE_CYCLES"]
    sq, ns = counters(src / "sq" / "run_counter_collection.csv", sqn, a.pmc_last)
    fetch_b = f["FETCH_SIZE"] * 1024 * 2  # KiB -> B, x2 gfx950 correction
    write_b = w["WRITE_SIZE"] * 1024
    out["pmc"] = {"dispatches_averaged": min(nf, nw, ns), "FETCH_SIZE_kib_raw": f["FETCH_SIZE"],
                  "WRITE_SIZE_kib": w["WRITE_SIZE"], "hbm_bytes_per_launch": fetch_b + write_b,
                  "GRBM_GUI_ACTIVE": f["GRBM_GUI_ACTIVE"], **sq}
    # issue-bound evidence: the share of wave cycles in which the wave issued an
    # instruction (SQ_* cycle counters are quad-cycles, both sides alike), VALU
    # instructions per wave, and the effective clock (GRBM_GUI_ACTIVE sums the 8 XCDs)
    waves = max(sq["SQ_WAVES"], 1.0)
    out["derived"] = {
        "issue_frac": sq["SQ_ACTIVE_INST_ANY"] / max(sq["SQ_WAVE_CYCLES"], 1.0),
        "valu_insts_per_wave": sq["SQ_INSTS_VALU"] / waves,
        "wave_cycles_per_wave": 4 * sq["SQ_WAVE_CYCLES"] / waves,
        "effective_clock_ghz": f["GRBM_GUI_ACTIVE"] / 8 / (out["avg_ms_rocprof"] * 1e-3) / 1e9,
    }
    if a.f64:  # executed FP64 VALU instructions per wave (x64 lanes: an upper bound on FP64 FLOP, FMA = 2)
        n64 = ["SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64"]
        c64, n6 = counters(src / "sq64" / "run_counter_collection.csv", n64, a.pmc_last)
        fl = 64 * (c64[n64[0]] + c64[n64[1]] + 2 * c64[n64[2]] + c64[n64[3]])
        out["pmc_f64"] = {**c64, "dispatches_averaged": n6, "fp64_flop_upper_bound_per_launch": fl,
                          "fp64_tflops_upper_bound": fl / (out["avg_ms_rocprof"] * 1e-3) / 1e12}
    if (src / "lanes").exists():  # VALU lane occupancy
        nl = ["SQ_INSTS_VALU_FLOPS_FP64", "SQ_INSTS_VALU_FLOPS_FP64_TRANS", "SQ_THREAD_CYCLES_VALU",
              "SQ_ACTIVE_INST_VALU"]
        cl, nn = counters(src / "lanes" / "run_counter_collection.csv", nl, a.pmc_last)
        # THREAD_CYCLES_VALU / ACTIVE_INST_VALU is the mean number of active lanes per VALU
        # instruction: 64.0 for torch's elementwise kernels and the perlin generator, 2.7 for a
        # one-thread kernel in the same passes (calibration).  SQ_INSTS_VALU_FLOPS_FP64
        # counts FLOPs per wave-instruction (1 add, 2 FMA), not per lane.
        lanes = {**cl, "dispatches_averaged": nn,
                 "valu_active_lanes": cl[nl[2]] / max(cl[nl[3]], 1.0)}
        lanes["valu_active_lane_frac"] = lanes["valu_active_lanes"] / 64.0
        if "pmc_f64" in out:  # the 64-lane bound scaled by the measured lane occupancy (all VALU alike)
            lanes["fp64_flop_active_lanes_per_launch"] = (out["pmc_f64"]["fp64_flop_upper_bound_per_launch"]
                                                          * lanes["valu_active_lane_frac"])
        out["pmc_lanes"] = lanes
    (Path(str(dst) + "_summary.json")).write_text(json.dumps(out, indent=1))
    print(json.dumps(out, indent=1))
    if a.traffic:  # the entry bench.py reads for a line of exactly this launch shape (profile_entry)
        tj = dst.parent / "traffic.json"
        cur = json.loads(tj.read_text()) if tj.exists() else {}
        cfg = bench["config"]
        prec, envs = cfg["precision"], cfg["envs_per_gpu"]
        spl = cfg.get("steps_per_launch", 1) if a.kernel in ("multi", "pair") else 1
        terrain = cfg.get("terrain") or cfg.get("workload", "").split(", ")[1].split(" ")[0]
        key = f"{prec}_{terrain}_n{envs}_spl{spl:g}"
        cur[key] = {
            "precision": prec, "envs": envs, "steps_per_launch": spl, "terrain": terrain,
            "bytes_per_launch": fetch_b + write_b, "fetch_raw_bytes_per_launch": f["FETCH_SIZE"] * 1024,
            "write_bytes_per_launch": write_b, "issue_frac": out["derived"]["issue_frac"],
            "avg_ms_rocprof": out["avg_ms_rocprof"],
            "fp64_flop_executed_per_launch": (out.get("pmc_f64") or {}).get("fp64_flop_upper_bound_per_launch"),
            "fp64_flop_active_lanes_per_launch": (out.get("pmc_lanes") or {}).get("fp64_flop_active_lanes_per_launch"),
            "source": str(dst) + "_summary.json"}
        tj.write_text(json.dumps(cur, indent=1))

if __name__ == "__main__":
    main()
