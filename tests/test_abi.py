"""The C-ABI boundary (include/ballbot_mi355x.h) without a GPU: the built
gfx950 library loads, exports every declared entry point, reports its ABI
version and fills default params; no compute call is made here."""
import ctypes as C
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
HEADER = ROOT / "include" / "ballbot_mi355x.h"


def _declared():
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|void|const char\*)\s+(bb_\w+)\s*\(", text, flags=re.M)))


@pytest.fixture(scope="module")
def native():
    from ballbot_gym import _native

    _native.build()  # no-op when up to date; hipcc cross-compiles for gfx950 without a GPU
    return _native


def test_header_declares_boundary():
    names = _declared()
    for must in ("bb_create", "bb_destroy", "bb_step", "bb_reset", "bb_set_hfield", "bb_assign_terrain",
                 "bb_get_state", "bb_set_state", "bb_forward", "bb_last_error", "bb_abi_version"):
        assert must in names


def test_library_exports_every_declared_symbol(native):
    lib = C.CDLL(str(native.LIB_PATH))
    missing = [n for n in _declared() if not hasattr(lib, n)]
    assert not missing, missing
    assert set(_declared()) == set(native.EXPORTS)


def test_abi_version_and_defaults(native):
    L = native.lib()
    assert L.bb_abi_version() == native.ABI_VERSION
    hdr = HEADER.read_text()
    assert f"#define BB_ABI_VERSION {native.ABI_VERSION}" in hdr
    p = native.default_params()
    assert (p.max_ep_steps, p.max_allowed_tilt, p.max_wheel_velocity) == (4000, 20.0, 10.0)
    assert abs(p.reward_scale - 0.01) < 1e-9 and abs(p.survival_bonus - 0.02) < 1e-9
    assert p.action_reg_coef == pytest.approx(-1e-4, rel=1e-6)
    assert (p.target_dir[0], p.target_dir[1]) == (0.0, 1.0)
    assert C.sizeof(native.BBParams) == C.sizeof(p)


def test_errors_are_reported_not_raised(native):
    """Invalid arguments return < 0 and set bb_last_error (no GPU touched)."""
    L = native.lib()
    assert L.bb_step(None, None, None, None, None, None, None, 0, None) < 0
    assert "NULL handle" in native.last_error()
    h = C.c_void_p()
    assert L.bb_create(0, 0, None, C.byref(h)) < 0
    assert "n_envs" in native.last_error()


def test_product_path_has_no_cpu_fallback(native, monkeypatch, tmp_path):
    """A missing HIP library is an error, never a silent CPU path."""
    monkeypatch.setattr(native, "_lib", None)
    monkeypatch.setattr(native, "LIB_PATH", tmp_path / "missing.so")
    with pytest.raises(native.NativeLibraryError):
        native.lib()


def _err(native):
    return native.last_error()


def test_argument_errors_without_gpu(native):
    """Invalid arguments are rejected before any HIP call: status < 0 and a
    bb_last_error message (the header's error contract), no crash."""
    L = native.lib()
    h = C.c_void_p()
    p = native.default_params()
    assert L.bb_create(0, 0, C.byref(p), C.byref(h)) < 0
    assert "n_envs must be > 0" in _err(native)
    p.n_terrains = 0
    assert L.bb_create(16, 0, C.byref(p), C.byref(h)) < 0
    assert "n_terrains" in _err(native)
    assert L.bb_create(16, 0, None, None) < 0 and "out is NULL" in _err(native)
    for call, msg in ((lambda: L.bb_step(None, None, None, None, None, None, None, 0, None), "NULL handle"),
                      (lambda: L.bb_reset(None, None, None, None), "NULL handle"),
                      (lambda: L.bb_set_hfield(None, 0, None, C.c_float(2.0)), "NULL handle"),
                      (lambda: L.bb_render_depth(None, None, None, 64, 64, 6, 0, None), "NULL argument"),
                      (lambda: L.bb_gae(None, None, None, None, None, 4, 4, 0.99, 0.95, None, None, None),
                       "NULL argument"),
                      (lambda: L.bb_ppo_loss(*([None] * 8), 8, 0, C.c_float(0.0), C.c_float(1.0), None, None, None,
                                             None), "NULL argument"),
                      (lambda: L.bb_generate_perlin(None, 0, 1, None, None, C.c_float(2.0)), "NULL argument"),
                      (lambda: L.bb_adamw_clip(None, None, None, None, 16, None, None, None, 0.9, 0.999, 1e-8, 0.01,
                                               0.5, None), "NULL argument"),
                      (lambda: L.bb_adamw_clip(16, 16, 16, 16, 0, 16, 16, 16, 0.9, 0.999, 1e-8, 0.01, 0.5, None),
                       "n must be >= 1"),
                      (lambda: L.bb_kernel_ms(None, None, None), "NULL argument"),
                      (lambda: L.bb_get_stats(None, None, 6), "NULL argument"),
                      (lambda: L.bb_ppo_mlp_act(16, (C.c_int32 * 21)(*([0] * 20 + [40000])), 40000, 16, 15, None, 4,
                                                None, 16, None, 16, 16, None), "inside the 40000-float buffer"),
                      (lambda: L.bb_set_terrain_stream(None, None, 1, 4, None), "NULL handle"),
                      (lambda: L.bb_get_env_terrain(None, None, None), "NULL handle"),
                      (lambda: L.bb_step_multi(None, None, 4, None, None, None, None, None, 1, None), "NULL handle"),
                      (lambda: L.bb_rollout(None, None, None), "NULL handle")):
        assert call() < 0
        assert msg in _err(native), (msg, _err(native))


def test_ctypes_structs_match_the_header(tmp_path, native):
    """The ctypes mirrors of the header's structs (bb_ppo_mlp_args, bb_encoder_params)
    have the C compiler's size and field offsets (gcc on the header, no GPU)."""
    import shutil
    import subprocess

    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    structs = {"bb_ppo_mlp_args": native.PPOMlpArgs, "bb_encoder_params": native.EncoderParams,
               "bb_params": native.BBParams, "bb_perlin_cfg": native.PerlinCfg, "bb_rollout_args": native.RolloutArgs}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "ballbot_mi355x.h"', 'int main(void) {']
    for cname, py in structs.items():
        lines.append(f'printf("{cname} size %zu\\n", sizeof({cname}));')
        for field, _ in py._fields_:
            lines.append(f'printf("{cname} {field} %zu\\n", offsetof({cname}, {field}));')
    lines += ["return 0;", "}"]
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", str(ROOT / "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    got = {tuple(line.split()[:2]): int(line.split()[2]) for line in out if line.strip()}
    for cname, py in structs.items():
        assert got[(cname, "size")] == C.sizeof(py), cname
        for field, _ in py._fields_:
            assert got[(cname, field)] == getattr(py, field).offset, (cname, field)
