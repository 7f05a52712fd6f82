"""CPU tier: the C-ABI library loads and exports every entry point include/poissbox_gpu.h declares;
host-only logic (slab partition) is checked without a GPU."""
import os
import re

import pytest

import poissbox_amd as pb
from poissbox_amd import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(REPO, "include", "poissbox_gpu.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pb_[a-z0-9_]+)\s*\(", src)) - {"pb_sendrecv_fn", "pb_allreduce_fn"})


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    names = header_functions()
    assert len(names) >= 40
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    # the Python binding declares a signature for each of them
    assert set(names) <= set(_lib.EXPORTED), set(names) - set(_lib.EXPORTED)


def test_version_and_error_string():
    lib = _lib.load()
    assert isinstance(lib.pb_last_error(), bytes)
    import ctypes as C
    a, b = C.c_int(), C.c_int()
    assert lib.pb_version(C.byref(a), C.byref(b)) == 0 and (a.value, b.value) == (0, 2)


@pytest.mark.parametrize("nz,nranks", [(64, 3), (7, 3), (1024, 8), (5, 5), (512, 1), (13, 4)])
def test_slab_partition(nz, nranks):
    parts = [pb.slab_partition(nz, nranks, r) for r in range(nranks)]
    assert parts[0][0] == 0
    for (k0, nk), (k1, _) in zip(parts, parts[1:]):
        assert k0 + nk == k1
    assert sum(nk for _, nk in parts) == nz
    sizes = [nk for _, nk in parts]
    assert max(sizes) - min(sizes) <= 1 and sizes == sorted(sizes, reverse=True)


def test_readme_dof_split():
    """README.md:30-32: 64^3 on 3 ranks -> 90112 / 86016 / 86016 DoF (22/21/21 planes)."""
    assert [pb.slab_partition(64, 3, r)[1] * 64 * 64 for r in range(3)] == [90112, 86016, 86016]


def test_bad_partition_raises():
    with pytest.raises(pb.PbError):
        pb.slab_partition(4, 2, 5)


def test_options_parse_petsc_names():
    o = pb.ksp_options(["-ksp_type", "cg", "-pc_type", "none", "-ksp_rtol", "1e-10",
                        "-ksp_max_it", "77", "-ksp_monitor", "-ksp_converged_reason", "-foo"])
    assert o.pc_type == pb.PC_NONE and o.rtol == 1e-10 and o.max_it == 77
    assert o.monitor == 1 and o.converged_reason == 1 and o.nullspace == 1
    d = pb.ksp_options()
    assert (d.rtol, d.atol, d.dtol, d.max_it, d.pc_type) == (1e-5, 1e-50, 1e5, 10000, pb.PC_JACOBI)
    with pytest.raises(pb.PbError):
        pb.ksp_options(["-ksp_type", "gmres"])
    assert d.cg_single_reduction == 0


def test_options_parse_single_reduction():
    """-ksp_cg_single_reduction (PetscOptionsBool: bare flag = true, or an explicit value)."""
    assert pb.ksp_options(["-ksp_cg_single_reduction"]).cg_single_reduction == 1
    o = pb.ksp_options(["-ksp_cg_single_reduction", "-ksp_rtol", "1e-9"])
    assert o.cg_single_reduction == 1 and o.rtol == 1e-9
    # PetscOptionsStringToBool: case-insensitive, on/off too (FALSE turned it on)
    for v, want in (("true", 1), ("1", 1), ("yes", 1), ("false", 0), ("0", 0), ("no", 0),
                    ("FALSE", 0), ("True", 1), ("on", 1), ("OFF", 0), ("No", 0), ("YES", 1)):
        o = pb.ksp_options(["-ksp_cg_single_reduction", v, "-ksp_max_it", "5"])
        assert o.cg_single_reduction == want and o.max_it == 5


def test_struct_layouts_match_header(tmp_path):
    """The ctypes mirrors of the header's structs have the C sizes and field offsets (gcc on
    include/poissbox_gpu.h): a stale mirror would let pb_ksp_opts_default write past it."""
    import ctypes as C
    import subprocess
    structs = {"pb_ksp_opts": _lib.KspOpts, "pb_ksp_result": _lib.KspResult}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "poissbox_gpu.h"',
             'int main(void) {']
    for cname, py in structs.items():
        lines.append(f'  printf("{cname} %zu\\n", sizeof({cname}));')
        for f in py._fields_:
            lines.append(f'  printf("{cname}.{f[0]} %zu\\n", offsetof({cname}, {f[0]}));')
    lines.append('  return 0; }')
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines) + "\n")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)],
                   check=True)
    got = dict(l.split() for l in subprocess.run([str(exe)], check=True, capture_output=True,
                                                 text=True).stdout.splitlines())
    for cname, py in structs.items():
        assert int(got[cname]) == C.sizeof(py), cname
        for f in py._fields_:
            assert int(got[f"{cname}.{f[0]}"]) == getattr(py, f[0]).offset, (cname, f[0])


def test_tuning_table_round_trip():
    """pb_tune_set / pb_tune_get / pb_tune_reset (host-only): set values read back, unset names
    report None (the launcher's measured default), unknown names are an error."""
    pb.tune_reset()
    assert pb.tune_get("cg_defer_x") is None
    pb.tune_set("cg_defer_x", 2)
    pb.tune_set("mg_engine_min_plane", 0)
    assert pb.tune_get("cg_defer_x") == 2 and pb.tune_get("mg_engine_min_plane") == 0
    with pytest.raises(pb.PbError):
        pb.tune_set("no_such_knob", 1)
    with pytest.raises(pb.PbError):
        pb.tune_get("PB_CG_DEFER_X")  # the environment spelling is not a tuning name
    pb.tune_reset()
    assert pb.tune_get("cg_defer_x") is None


def test_library_reads_only_the_documented_environment():
    """The product library's getenv sites name only the user settings INTEGRATION.md lists (plus
    the launcher's rank variables): kernel variants are tuning-table entries, not environment
    knobs."""
    csrc = os.path.join(REPO, "poissbox_amd", "csrc")
    names = set()
    for f in os.listdir(csrc):
        if f.endswith((".hip", ".cpp", ".hpp")):
            src = open(os.path.join(csrc, f)).read()
            names |= set(re.findall(r'(?:getenv|env_int)\("(PB_[A-Z0-9_]+)"', src))
    documented = {"PB_COMM_TIMEOUT_MS", "PB_DEVICE", "PB_TRANSPORT", "PB_SHM_SLOT_DOUBLES",
                  "PB_RENDEZVOUS_DIR", "PB_RENDEZVOUS_SLACK_S", "PB_ROCTX"}
    assert names <= documented, names - documented
    integ = open(os.path.join(REPO, "INTEGRATION.md")).read()
    assert all(f"`{n}" in integ for n in documented)


def test_every_tuning_name_is_documented():
    """Every name of the library's tuning table (pb_runtime.cpp kTuneNames) has a row in
    INTEGRATION.md's tuning table, and the table lists no name the library does not know."""
    src = open(os.path.join(REPO, "poissbox_amd", "csrc", "pb_runtime.cpp")).read()
    i = src.index("kTuneNames[] = {")
    names = set(re.findall(r'"([a-z0-9_]+)"', src[i:src.index("};", i)]))
    assert len(names) >= 20
    integ = open(os.path.join(REPO, "INTEGRATION.md")).read()
    table = integ[integ.index("## Tuning table"):]
    missing = sorted(n for n in names if f"`{n}`" not in table)
    assert not missing, missing
    for n in names:
        pb.tune_set(n, pb.tune_get(n) or 0)  # known to the library
    pb.tune_reset()
