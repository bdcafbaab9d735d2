"""Run bench.py against a variant build of the HIP library (diagnostic A/B, GPU box).

  python tools/bench_with_lib.py tools/_build/libbb_<name>.so [bench.py args ...]
"""
import runpy
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "openballbot-rl_amd"))

import torch  # noqa: E402,F401  (torch's HIP runtime first, as in bench.py)
from ballbot_gym import _native  # noqa: E402

_native.use_diagnostic_library(Path(sys.argv[1]).resolve())
sys.argv = [str(ROOT / "bench.py")] + sys.argv[2:]
runpy.run_path(str(ROOT / "bench.py"), run_name="__main__")
