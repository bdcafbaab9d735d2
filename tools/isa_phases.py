"""Static instruction counts per solver phase (tool, not shipped).

Counts the instructions of each kernel's solve16 between the `; PHASE_MARK k`
comments that a -DBB_ISA_MARKS build leaves in the assembly (bb_solve.h: PH).
Static counts: a loop body counts once, so the line-search loop (phase 9) is
one evaluation and the contact loops one round.

  hipcc --offload-arch=gfx950 -O3 -std=c++17 -DBB_ISA_MARKS -I openballbot-rl_amd/csrc \
      --cuda-device-only -S -o /tmp/bbk.s openballbot-rl_amd/csrc/bb_kernels.hip
  python tools/isa_phases.py /tmp/bbk.s
"""
import re
import sys
from collections import Counter

NAMES = {0: "contact pass", 1: "ground sums", 2: "gradient", 3: "hessian row", 4: "cholesky",
         5: "sweeps", 8: "ls setup", 9: "ls loop", 6: "update", 7: "exit"}


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if "_dpp" in op or op.startswith("v_mov_b32_dpp"):
        return "dpp"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main(path):
    func, marks, counts = None, [], {}
    cur = None
    for line in open(path):
        m = re.match(r"^(_Z[^:\s]+):", line)
        if m:
            func, cur = m.group(1), None
            continue
        m = re.search(r"; PHASE_MARK (\d+)", line)
        if m and func:
            cur = int(m.group(1))
            if cur == 7:  # solver exit: the rest of the kernel is not the solve
                cur = None
                continue
            counts.setdefault(func, {}).setdefault(cur, Counter())
            continue
        s = line.strip()
        if cur is None or not s or s.startswith((";", ".")) or s.endswith(":"):
            continue
        op = s.split()[0]
        counts[func][cur][classify(op)] += 1
    for func, ph in counts.items():
        print(func[:90])
        tot = Counter()
        order = [10, 0, 1, 2, 3, 4, 5, 8, 9, 6]  # PH(k) ends phase k; code after mark k is the next phase
        for k in order:
            if k not in ph:
                continue
            c = ph[k]
            nxt = {10: "contact pass", 0: "ground sums", 1: "gradient", 2: "hessian row", 3: "cholesky", 4: "sweeps",
                   5: "ls setup", 8: "ls loop", 9: "update", 6: "conv test"}[k]
            tot.update(c)
            print("  after mark %d (%-14s) valu %5d dpp %4d lds %4d vmem %3d salu %4d wait %4d" %
                  (k, nxt, c["valu"], c["dpp"], c["lds"], c["vmem"], c["salu"], c["wait"]))
        print("  total                        valu %5d dpp %4d lds %4d vmem %3d salu %4d wait %4d" %
              (tot["valu"], tot["dpp"], tot["lds"], tot["vmem"], tot["salu"], tot["wait"]))


if __name__ == "__main__":
    main(sys.argv[1])
