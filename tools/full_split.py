"""Per-launch durations of the step kernels from a rocprofv3 kernel_trace.csv:
the fast kernel, and the full kernel's two launches per step (the predicted
list on the side stream, then the hand-overs), told apart by launch order."""
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
fast, full_pred, full_hand, step = [], [], [], []
seen_full = 0
last_pred_start = None
for r in rows:
    n = r["Kernel_Name"]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    if "step_kernel" in n and ", false>" in n:
        fast.append(d)
    elif "step_kernel" in n and ", true>" in n:
        (full_pred if seen_full % 2 == 0 else full_hand).append(d)
        seen_full += 1
    elif "predict_kernel" in n:
        if last_pred_start is not None:
            step.append((int(r["Start_Timestamp"]) - last_pred_start) / 1e6)
        last_pred_start = int(r["Start_Timestamp"])
for name, v in (("fast", fast), ("full_predicted", full_pred), ("full_handover", full_hand), ("predict->predict", step)):
    if v:
        v = v[len(v) // 3:]  # skip warmup
        print(f"{name:18s} n={len(v):4d} mean={statistics.mean(v):.3f} ms median={statistics.median(v):.3f} max={max(v):.3f}")
