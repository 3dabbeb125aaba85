"""The float64 quad miscompile's bug class, checked on the ISA.

Round 5's default-schedule build of team_step_kernel<F64<Ant>,16> copied two live-through doubles
into AGPRs inside a divergent region's join block, before the `s_or_b64 exec, exec, sN` that restores
the region's lanes; lanes outside the region then read stale registers (found on the GPU by
register-file poisoning, tools/vgpr_poison_probe.py).  tools/isa_uninit.py --exec-copies flags that
pattern; these tests pin the checker on a synthetic reproducer and run it over the product's float64
quad kernels compiled from this tree.  CPU only (hipcc cross-compiles gfx950).
"""
import os
import shutil
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
import isa_uninit  # noqa: E402

KERNEL = "_Z6kernelv"
FAULTY = f"""{KERNEL}:                  ; @{KERNEL}
; %bb.0:
	v_mov_b32_e32 v240, v1
	v_mov_b32_e32 v241, v2
	v_cmp_gt_f64_e32 vcc, 0, v[4:5]
	s_and_saveexec_b64 s[18:19], vcc
	s_cbranch_execz .LBB0_2
; %bb.1:
	v_add_f64 v[6:7], v[6:7], v[240:241]
.LBB0_2:
	v_accvgpr_write_b32 a54, v240
	v_accvgpr_write_b32 a55, v241
	s_or_b64 exec, exec, s[18:19]
	v_accvgpr_read_b32 v8, a54
	v_accvgpr_read_b32 v9, a55
	v_add_f64 v[6:7], v[6:7], v[8:9]
	s_endpgm
.Lfunc_end0:
"""
# the same copies after the EXEC restore (every lane copies): correct code
FIXED = FAULTY.replace("""	v_accvgpr_write_b32 a54, v240
	v_accvgpr_write_b32 a55, v241
	s_or_b64 exec, exec, s[18:19]
""", """	s_or_b64 exec, exec, s[18:19]
	v_accvgpr_write_b32 a54, v240
	v_accvgpr_write_b32 a55, v241
""")
# a value computed inside the region and copied there is the region's own business (not flagged)
INSIDE = FAULTY.replace("""; %bb.1:
	v_add_f64 v[6:7], v[6:7], v[240:241]
""", """; %bb.1:
	v_add_f64 v[240:241], v[6:7], v[240:241]
""")

# the spill form: a live-through value stored to a scratch slot under the region's EXEC, reloaded after
SPILL = FAULTY.replace("""	v_accvgpr_write_b32 a54, v240
	v_accvgpr_write_b32 a55, v241
	s_or_b64 exec, exec, s[18:19]
	v_accvgpr_read_b32 v8, a54
	v_accvgpr_read_b32 v9, a55
""", """	scratch_store_dwordx2 off, v[240:241], off offset:16 ; 8-byte Folded Spill
	s_or_b64 exec, exec, s[18:19]
	scratch_load_dwordx2 v[8:9], off, off offset:16 ; 8-byte Folded Reload
""")


def _check(tmp_path, text):
    p = tmp_path / "k.s"
    p.write_text(text)
    return isa_uninit.exec_copies(isa_uninit.parse(str(p), KERNEL))


def test_checker_flags_the_round5_pattern(tmp_path):
    hits = _check(tmp_path, FAULTY)
    assert [h[1] for h in hits] == ["v_accvgpr_write_b32 a54, v240", "v_accvgpr_write_b32 a55, v241"]


def test_checker_flags_the_spill_form(tmp_path):
    hits = _check(tmp_path, SPILL)
    assert len(hits) == 1 and hits[0][1].startswith("scratch_store_dwordx2 off, v[240:241]")


def test_checker_passes_copies_after_the_exec_restore(tmp_path):
    assert _check(tmp_path, FIXED) == []
    assert _check(tmp_path, INSIDE) == []


@pytest.mark.timeout(900)
@pytest.mark.skipif(shutil.which("/opt/rocm/bin/hipcc") is None, reason="hipcc absent")
@pytest.mark.parametrize("robot", ["Ant", "AntMuJoCo"])
def test_product_float64_quad_kernel_has_no_partial_exec_copies(tmp_path, robot):
    """The product's float64 quad translation unit (Makefile T64FLAGS), compiled from this tree."""
    out = tmp_path / f"team64_{robot}.s"
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fno-slp-vectorize",
                           "-DPBG_TEAM64_TU", f"-DPBG_ROBOT={robot}", "--cuda-device-only", "-S", "-o", str(out),
                           os.path.join(REPO, "pybullet-gym_amd", "csrc", "pbg_robot.hip")],
                          stderr=subprocess.DEVNULL)
    names = [k for k in isa_uninit.kernels(str(out)) if "team_step_kernel" in k]
    assert names, "no quad kernel in the ISA"
    for k in names:
        assert isa_uninit.exec_copies(isa_uninit.parse(str(out), k)) == [], k


@pytest.mark.timeout(900)
@pytest.mark.skipif(shutil.which("/opt/rocm/bin/hipcc") is None or not os.path.isdir(os.path.join(REPO, ".git")),
                    reason="needs hipcc and the git history")
def test_round5_source_reproduces_the_faulting_copies(tmp_path):
    """The real instance: the round-5 source (commit 4428492) on the default schedule has the split
    copies of a54 / a55 / a180 / a181 before the region's EXEC restore -- the registers the GPU
    register-file bisection found (profiles/r06_f64_quad_miscompile/register_bisect.txt) -- and the
    trackers build it shipped with has none (tools/repro_r05_miscompile.sh)."""
    out = subprocess.run(["bash", os.path.join(REPO, "tools", "repro_r05_miscompile.sh"), str(tmp_path / "w")],
                         capture_output=True, text=True, timeout=800).stdout
    default, trackers = out.split("trackers.s:")
    for reg in ("a54, v", "a55, v", "a180, v", "a181, v"):
        assert f"v_accvgpr_write_b32 {reg}" in default, (reg, out)
    assert trackers.strip().startswith("0 copies"), out
