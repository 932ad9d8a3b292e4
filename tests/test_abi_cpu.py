"""CPU-side checks of the boundary: libhz.so loads and exports every symbol
declared in include/hz_abi.h; the record packer round-trips every golden
state.  No GPU calls."""
import os
import re
import subprocess

import numpy as np

from conftest import GOLDEN, PKG, ROOT
from hzamd.state import pack_ref, unpack_ref, ref_from_object, apply_ref_to_object


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "hz_abi.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(hz_[a-z_0-9]+)\s*\(", src)))


def test_header_symbols_exported_by_libhz():
    lib = os.path.join(PKG, "libhz.so")
    assert os.path.exists(lib), "run __graft_entry__.build() first"
    out = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True, text=True, check=True).stdout
    exported = set(l.split()[-1] for l in out.splitlines() if l.strip())
    missing = [s for s in declared_symbols() if s not in exported]
    assert not missing, missing


def test_python_binding_covers_header():
    import hzamd._native as nat
    assert sorted(nat.exported_symbols()) == declared_symbols()


def test_libhz_loads_without_gpu():
    import hzamd._native as nat
    L = nat.lib()
    assert L.hz_version().startswith(b"hz ")
    assert L.hz_env_size(None) == -1


def test_libhz_targets_gfx950():
    data = open(os.path.join(PKG, "libhz.so"), "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data


def test_pack_roundtrip_all_golden_states():
    f = np.load(os.path.join(GOLDEN, "env_traces.npz"))
    for v in list(f["states"]) + list(f["finals"]):
        assert (unpack_ref(pack_ref(v)) == v).all()


def test_object_roundtrip():
    f = np.load(os.path.join(GOLDEN, "env_traces.npz"))

    class G:
        pass
    for v in f["states"][::37]:
        g = apply_ref_to_object(v, G())
        assert (ref_from_object(g) == v).all()


def test_tower_class_table_is_bank_conflict_free():
    """csrc/hz_net.hip's kX6ClassRow equals tools/class_table.py's generated
    table, whose A-fragment ds_read_b128s (every tap, plane and row block of
    a chunk, the corner rows' zero-region redirects and the padding rows'
    wildcard reads included) and staging stores take exactly the
    conflict-free LDS cycles (MI355X_MICROARCH.md's lane groups and banks)."""
    import subprocess
    import sys
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "class_table.py")], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "source table equals it" in r.stdout and "(1584, 1584)" in r.stdout
