"""Register / LDS / scratch metadata of every kernel in the HIP sources (CPU, no GPU).

python tools/kernel_regs.py [--out profiles/r03_kernel_registers.json]

Compiles each csrc/*.hip device-only for gfx950 (the same flags as the product
build) and reads the AMDGPU code-object notes (llvm-readelf --notes).  On
gfx950's unified register file `.vgpr_count` already includes the AGPRs
(`.agpr_count` of them); a SIMD holds floor(512 / alloc) waves of a kernel,
alloc = vgpr_count rounded up to the 8-register granule.  rocprofv3's
kernel-trace "VGPR" column reads alloc / 2 for these kernels (e.g. 184 for the
366-register fast fp64 step kernel), which is why it disagreed with the notes.
"""
from __future__ import annotations

import argparse
import json
import re
import subprocess
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "openballbot-rl_amd" / "csrc"
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"
KEYS = ("vgpr_count", "agpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count",
        "private_segment_fixed_size", "group_segment_fixed_size")


def demangle(names):
    r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
    return r.stdout.splitlines() if r.returncode == 0 else names


def kernels_of(src: Path, tmp: Path) -> list[dict]:
    co = tmp / (src.stem + ".co")
    import sys
    sys.path.insert(0, str(ROOT / "openballbot-rl_amd"))
    from ballbot_gym._native import SOURCE_FLAGS

    subprocess.run(["hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only",
                    "--no-gpu-bundle-output", *SOURCE_FLAGS.get(src.name, []), "-c", str(src), "-o", str(co)],
                   check=True)
    notes = subprocess.run([READELF, "--notes", str(co)], check=True, capture_output=True, text=True).stdout
    out, cur, col = [], None, -1
    for line in notes.splitlines():
        m = re.match(r"(\s*(?:-\s+)?)\.(\w+):\s+(\S+)", line)
        if not m:
            continue
        if m.group(2) == "agpr_count" and "-" in m.group(1):  # a kernel record (its keys are sorted, this one first)
            cur, col = {}, len(m.group(1))
            out.append(cur)
        if cur is not None and len(m.group(1)) == col and m.group(2) in KEYS + ("name",):
            cur[m.group(2)] = m.group(3) if m.group(2) == "name" else int(m.group(3))
    ks = [k for k in out if "name" in k and "vgpr_count" in k and not k["name"].endswith(".kd")]
    for k, d in zip(ks, demangle([k["name"] for k in ks])):
        k["kernel"] = d
        alloc = -(-k["vgpr_count"] // 8) * 8
        k["vgpr_alloc"] = alloc
        k["waves_per_simd_by_vgpr"] = 512 // alloc if alloc else 8
        k["rocprof_vgpr_field"] = alloc // 2
        k["source"] = src.name
    return ks


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=str(ROOT / "profiles" / "r03_kernel_registers.json"))
    a = ap.parse_args()
    res = []
    with tempfile.TemporaryDirectory() as t:
        for src in sorted(CSRC.glob("*.hip")):
            res += kernels_of(src, Path(t))
    Path(a.out).write_text(json.dumps({"what": __doc__.strip().splitlines()[0], "kernels": res}, indent=1) + "\n")
    for k in res:
        print(f"{k['vgpr_count']:4d} vgpr ({k['agpr_count']:3d} agpr) {k['private_segment_fixed_size']:5d} B scratch "
              f"{k['group_segment_fixed_size']:6d} B lds  {k['kernel'][:110]}")


if __name__ == "__main__":
    main()
