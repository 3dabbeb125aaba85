"""Model compiler: committed tables current, mass properties sane, topology as expected."""
import json
import os

import numpy as np
import pytest

import pybulletgym_amd  # noqa: F401
from pybulletgym_amd import codegen, mjcf, robots

REF_ASSETS = robots.reference_asset_dir()


@pytest.mark.skipif(not os.path.isdir(REF_ASSETS), reason="reference assets only in the build container")
def test_committed_tables_are_current():
    tables = codegen.compile_all()
    with open(codegen.HEADER) as f:
        assert f.read() == codegen.emit_header(tables), "run python -m pybulletgym_amd.codegen"
    for key, t in tables.items():
        assert codegen.load_tables(key)["NL"] == t["NL"]


@pytest.mark.parametrize("key", list(robots.SPECS))
def test_table_invariants(key):
    t = codegen.load_tables(key)
    spec = robots.spec_for(key)
    assert t["NA"] == spec.action_dim
    if spec.kind == robots.KIND_WALKER:
        assert t["OBS"] == 8 + 2 * t["NO"] + t["NF"]  # robot_locomotors.py:60-64
    for l, I in enumerate(t["link_inertia"]):
        M = np.array([[I[0], I[3], I[4]], [I[3], I[1], I[5]], [I[4], I[5], I[2]]])
        ev = np.linalg.eigvalsh(M)
        assert ev.min() >= -1e-12, (key, l)
        if t["link_mass"][l] > 0:
            assert ev.min() > 0
    for p in t["link_parent"]:
        assert p < len(t["link_parent"])
    assert all(p < i for i, p in enumerate(t["link_parent"]))  # parents before children


def test_ant_topology():
    t = codegen.load_tables("ant")
    assert t["floating"] == 1 and t["NL"] == 12 and t["NJ"] == 8 and t["NDOF"] == 14
    # MJCF depth-first joint order, not the <actuator> order (ant.xml:61-70)
    assert t["act_joint_names"] == ["hip_1", "ankle_1", "hip_2", "ankle_2", "hip_3", "ankle_3", "hip_4", "ankle_4"]
    assert t["act_gain"] == [250.0] * 8  # power 2.5 * power_coef 100
    assert t["NS"] == 25  # torso sphere + 12 capsules x 2 endpoints
    assert t["base_pos"] == [0.0, 0.0, 0.75]


def test_halfcheetah_mass_and_gains():
    t = codegen.load_tables("halfcheetah")
    assert abs(sum(t["link_mass"]) + t["base_mass"] - 14.0) < 1e-9  # settotalmass="14"
    assert t["act_gain"] == pytest.approx([0.9 * c for c in (120, 90, 60, 140, 60, 30)])


def test_humanoid_dummies_and_pairs():
    t = codegen.load_tables("humanoid")
    assert t["NJ"] == 17 and t["NL"] == 19
    assert t["initial_z_fixed"] == 0.8
    assert t["NPAIR"] > 0
    names = t["link_name"]
    for a, b in zip(t["pair_link_a"], t["pair_link_b"]):
        # never an ancestor pair (URDF_USE_SELF_COLLISION_EXCLUDE_ALL_PARENTS)
        def anc(i):
            out = []
            while t["link_parent"][i] >= 0:
                i = t["link_parent"][i]
                out.append(i)
            return out
        assert a not in anc(b) and b not in anc(a), (names[a], names[b])


def test_walker2d_topology_and_gains():
    """robot_locomotors.py:93-106: power 0.40, foot joints power_coef 30 (robot_specific_reset)."""
    t = codegen.load_tables("walker2d")
    assert t["floating"] == 0 and t["NJ"] == 9 and t["NA"] == 6 and t["OBS"] == 22
    assert t["act_joint_names"] == ["thigh_joint", "leg_joint", "foot_joint",
                                    "thigh_left_joint", "leg_left_joint", "foot_left_joint"]
    assert t["act_gain"] == pytest.approx([40.0, 40.0, 12.0, 40.0, 40.0, 12.0])
    assert [t["link_name"][l] for l in t["foot_link"]] == ["foot", "foot_left"]
