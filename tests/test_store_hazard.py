"""The compiled kernels leave two wait states between every store of more than 8 bytes and a VALU
rewrite of its data registers (tools/store_hazard_audit.py).  Without them gfx950 stored boards
whose first word was already overwritten by the next instruction (k_rollout_lean at 1M+ boards,
under store-queue back-pressure; tests/test_fullsize_gpu.py::test_rollout_large_n_vs_oracle).
CPU-only: hipcc cross-compiles the library's HIP sources to gfx950 assembly."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "reinforcement-learning-2048_amd", "csrc")
sys.path.insert(0, os.path.join(ROOT, "tools"))


@pytest.mark.skipif(shutil.which("hipcc") is None, reason="hipcc not in this image")
@pytest.mark.timeout(900)
def test_no_store_data_hazard(tmp_path):
    import store_hazard_audit

    out = []
    for f in audited_sources():
        s = str(tmp_path / (f + ".s"))
        subprocess.run(audit_cmd(os.path.join(CSRC, f), s), check=True, capture_output=True)
        out.append(s)
    assert sum(store_hazard_audit.audit(s) for s in out) == 0


def audited_sources():
    """Exactly the sources the shipped library is built from (__graft_entry__.SRCS)."""
    sys.path.insert(0, ROOT)
    import __graft_entry__ as G
    return list(G.SRCS)


def audit_cmd(src: str, out: str) -> list:
    """The library's own hipcc flags for this source (__graft_entry__.src_flags: HIPFLAGS --
    kernarg preloading changes the kernels' prologues, register allocation and scheduling -- and
    the source's own, e.g. g2048.hip's machine scheduler), minus the link-only ones, plus
    device-only assembly output: the audit reads the code that ships."""
    sys.path.insert(0, ROOT)
    import __graft_entry__ as G
    flags = [f for f in G.src_flags(src) if f not in ("-shared", "-fPIC")]
    return [G.HIPCC, *flags, "--cuda-device-only", "-S", src, "-o", out]


def test_audit_uses_library_flags():
    """A change of the library's build flags cannot silently move the audit off the shipped code
    (kernarg preloading was on in the library but not in the audit)."""
    sys.path.insert(0, ROOT)
    import __graft_entry__ as G
    cmd = audit_cmd("x.hip", "x.s")
    for f in G.HIPFLAGS:
        if f not in ("-shared", "-fPIC"):
            assert f in cmd
    assert "-amdgpu-kernarg-preload-count=16" in cmd
    assert set(audited_sources()) == set(G.SRCS)
    for src, extra in G.SRC_FLAGS.items():  # a source's own flags reach its audit too
        cmd = audit_cmd(os.path.join(CSRC, src), "x.s")
        assert all(f in cmd for f in extra), src


def test_audit_sees_loads_and_branches(tmp_path):
    """The audit sees every VGPR writer and follows branches: VALU writers count as hazards, LDS /
    VMEM load writers are notes."""
    import store_hazard_audit

    cases = {
        "valu": ("buffer_store_dwordx4 v[4:7], v1, s[0:3], 0 offen\n"
                 "v_mov_b32 v5, 0\n", 1),
        "lds": ("buffer_store_dwordx4 v[4:7], v1, s[0:3], 0 offen\n"
                "ds_read_b128 v[6:9], v2\n", 0),
        "vmem": ("global_store_dwordx4 v[0:1], v[4:7], off\n"
                 "global_load_dword v7, v[0:1], off\n", 0),
        "nop": ("buffer_store_dwordx4 v[4:7], v1, s[0:3], 0 offen\n"
                "s_nop 1\nv_mov_b32 v5, 0\n", 0),
        "branch": ("buffer_store_dwordx4 v[4:7], v1, s[0:3], 0 offen\n"
                   "s_branch .LBB0_2\nv_mov_b32 v5, 0\n.LBB0_2:\nv_mov_b32 v4, 0\n", 1),
        "cbranch": ("buffer_store_dwordx4 v[4:7], v1, s[0:3], 0 offen\n"
                    "s_cbranch_scc1 .LBB0_3\nv_mov_b32 v1, 0\ns_endpgm\n.LBB0_3:\n"
                    "v_add_u32 v6, v6, v6\n", 1),
        "other": ("buffer_store_dwordx4 v[4:7], v1, s[0:3], 0 offen\n"
                  "v_mov_b32 v8, 0\nds_read_b32 v3, v2\n", 0),
    }
    for name, (asm, want) in cases.items():
        p = tmp_path / (name + ".s")
        p.write_text("_Z1kv:\n" + asm)
        notes = []
        assert store_hazard_audit.audit(str(p), notes) == want, name
        assert len(notes) == (name in ("lds", "vmem")), name
