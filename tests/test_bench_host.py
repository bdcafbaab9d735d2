"""bench.py host logic (CPU): the algorithmic-byte model behind roofline.achieved
and the launch chunking of the multi-step bench."""
import sys
from pathlib import Path

import pytest

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402


def test_algorithmic_bytes_one_step_per_launch():
    # fp64 909 B per env-step (state r/w 752, action 12, obs 60, reward 4, done 1,
    # terminal obs 60, pos2d 8, step counter r/w 8, terrain id 4); fp32 533 B; relief terrain
    # + the 7 x 7 float32 hfield vertices under the ball (+196 B)
    assert bench.algorithmic_bytes("fp64") == 909
    assert bench.algorithmic_bytes("fp32") == 533
    assert bench.algorithmic_bytes("fp64", 1, relief=True) == 909 + 196


@pytest.mark.parametrize("k", [2, 20, 64, 256])
def test_algorithmic_bytes_multi_step_moves_state_once(k):
    per_launch = 2 * 47 * 8 + 8 + 4
    assert bench.algorithmic_bytes("fp64", k) == pytest.approx(per_launch / k + 145)
    # K steps of one env in one launch move less than K single-step launches
    assert k * bench.algorithmic_bytes("fp64", k) < k * bench.algorithmic_bytes("fp64")


@pytest.mark.parametrize("count,m,pool", [(500, 256, 256), (500, 64, 256), (20, 256, 256), (700, 200, 256),
                                          (1, 1, 256), (513, 256, 256)])
def test_launch_chunks_cover_the_steps_within_the_pool(count, m, pool):
    ch = bench.launch_chunks(count, m, pool)
    assert sum(ch) == count
    assert all(1 <= k <= m for k in ch)
    j = 0
    for k in ch:  # no launch reads past the end of the action pool
        assert j % pool + k <= pool
        j += k


def test_launch_chunks_bench_defaults_time_one_launch():
    """bench.py's defaults (512-slot action pool, 512 steps per launch): the 500 timed steps are
    one launch; burn-in + warm-up (700 steps) are 512 + 188."""
    assert bench.launch_chunks(500, 512, 512) == [500]
    assert bench.launch_chunks(700, 512, 512) == [512, 188]
    assert bench.launch_chunks(20, 512, 512) == [20]


def test_launch_chunks_driver_window_is_one_launch():
    # the driver's --steps 20 --warmup 5: one 20-step launch
    assert bench.launch_chunks(20, 256, 256) == [20]
    assert bench.launch_chunks(500, 256, 256) == [256, 244]


def test_committed_flops_and_profiles_name_their_basis():
    """Lines without the CPU leg (N > 1 ranks, --no-cpu-baseline) take the committed FLOP count of
    their terrain, on the same yardstick as the live count (bench.FLOP_BASIS); the same-shape
    profiles that roofline.traffic / frac_executed read exist for the driver's and the bench's
    flat launches and the perlin pair."""
    import json

    for t in ("flat", "perlin"):
        fl = bench.committed_flops(t)
        assert fl and fl["flops_per_env_step"] > 0 and fl["basis"] == bench.FLOP_BASIS
    tab = bench.ROOT / "profiles" / "traffic.json"
    for shape in (("flat", 20.0), ("flat", 500.0), ("perlin", 500.0)):
        e = bench.profile_entry(tab, "fp64", shape[0], 4096, shape[1])
        assert e.get("fp64_flop_active_lanes_per_launch", 0) > 0 and e.get("bytes_per_launch", 0) > 0, shape
        assert (bench.ROOT / e["source"]).exists(), e["source"]
    assert json.loads((bench.ROOT / "profiles" / "flops.json").read_text())
