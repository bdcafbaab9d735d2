"""Host build of the product's geometry templates (tests/hostcheck, CPU only).

- The base-tree contact's world form (bb_physics.h:BodyFrame, body_V), which the
  full kernel broadcasts instead of the 13-column Jacobian: J x = F V(x) against
  the Jacobian written column by column, for random contacts, poses and x.
- The separated capsule-prism distance (bb_bodycon.h:capsule_prism_apart: 9
  edge pairs + 10 face projections) against the minimum over the prism's 8
  boundary triangles, the oracle's form (oracle/bb_oracle.c: capsule_prism).
  tools/capsule_check.hip runs the same comparison on the GPU.
"""
import ctypes as C

import pytest

import hostcheck_lib as H


@pytest.fixture(scope="module")
def hc():
    return H.lib()


def test_body_contact_world_form_matches_jacobian(hc):
    assert hc.hc_body_jacobian_check(20000, 7) < 1e-13


def test_capsule_separation_distance_matches_triangle_form(hc):
    worst = C.c_double()
    mism = hc.hc_capsule_apart_check(200000, 11, C.byref(worst))
    assert mism == 0
    assert worst.value < 1e-9
