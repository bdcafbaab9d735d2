"""Run GPU tests against a variant build (diagnostic, GPU box).

  python tools/variant_test.py tools/_build/libbb_X.so <pytest args...>
"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "openballbot-rl_amd"))

if __name__ == "__main__":
    import torch  # noqa: F401  (the HIP runtime comes up through torch first, as in the tests)
    from ballbot_gym import _native

    _native.use_diagnostic_library(Path(sys.argv[1]).resolve())
    import pytest

    sys.exit(pytest.main(sys.argv[2:]))
