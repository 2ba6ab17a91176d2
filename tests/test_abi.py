"""CPU: the drop-in boundary.  The C-ABI library loads without a GPU, exports every
symbol include/*.h declares, and its instance structs have the reference's byte layout.
No compute call is made here (no GPU in this container)."""
import ctypes as C
import json
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "include")


def _declared_symbols():
    """Functions and objects declared by include/*.h, after the preprocessor expands the
    table/instance declaration macros."""
    names = set()
    for h in ("arm_math.h", "arm_math_mi355x.h", "arm_common_tables.h", "arm_const_structs.h"):
        out = subprocess.run(["gcc", "-E", "-P", "-I" + INC, os.path.join(INC, h)], capture_output=True,
                             text=True, check=True).stdout
        flat = " ".join(out.split())
        for decl in flat.split(";"):
            decl = decl.strip()
            if decl.startswith("typedef") or "{" in decl or "}" in decl:
                decl = decl.split("}")[-1].strip()
                if not decl or decl.startswith("typedef"):
                    continue
            m = re.search(r"\b((?:arm|twiddle|armBitRev)\w*)\s*\(", decl)
            if m and not decl.startswith("typedef"):
                names.add(m.group(1))
                continue
            m = re.search(r"^extern const [\w ]+?\b((?:arm|twiddle)\w*)\s*(\[|$)", decl)
            if m:
                names.add(m.group(1))
    return names


def test_library_exports_every_declared_symbol(dsp):
    names = _declared_symbols()
    assert len(names) >= 317, len(names)         # functions + data symbols, macro-expanded
    missing = []
    for n in sorted(names):
        try:
            getattr(dsp.lib, n)
        except AttributeError:
            missing.append(n)
    assert not missing, missing


def test_struct_layout_matches_reference():
    """tools/abi_layout.c compiled against include/ must print what it printed when
    compiled against the reference headers (tests/golden/abi_layout.json)."""
    exe = os.path.join(ROOT, "oracle", "_build", "abi_layout_ours")
    os.makedirs(os.path.dirname(exe), exist_ok=True)
    subprocess.run(["gcc", "-I" + INC, os.path.join(ROOT, "tools", "abi_layout.c"), "-o", exe], check=True)
    ours = json.loads(subprocess.run([exe], capture_output=True, text=True, check=True).stdout)
    ref = json.load(open(os.path.join(ROOT, "tests", "golden", "abi_layout.json")))
    assert ours == ref


def test_ctypes_mirror_matches_headers(dsp):
    from cmsisdsp_amd import _abi
    ref = json.load(open(os.path.join(ROOT, "tests", "golden", "abi_layout.json")))
    for name in ("arm_cfft_instance_f32", "arm_rfft_fast_instance_f32", "arm_fir_instance_f32",
                 "arm_fir_instance_q15", "arm_matrix_instance_f32", "arm_mfcc_instance_f32",
                 "arm_matrix_instance_q15", "arm_matrix_instance_q31", "arm_fir_instance_q31",
                 "arm_rfft_instance_q31", "arm_rfft_instance_q15"):
        st = getattr(_abi, name)
        assert C.sizeof(st) == ref[name]["size"], name
        for fname, _ in st._fields_:
            assert getattr(st, fname).offset == ref[name][fname], (name, fname)


def test_const_instances_point_at_exported_tables(dsp):
    """arm_cfft_sR_f32_len1024 = {1024, twiddleCoef_1024, armBitRevIndexTable1024, 1800}
    (arm_const_structs.c:104-106) — host-side data only, no device access."""
    S = dsp.const_instance("arm_cfft_sR_f32_len1024")
    tw = C.addressof(C.c_float.in_dll(dsp.lib, "twiddleCoef_1024"))
    br = C.addressof(C.c_uint16.in_dll(dsp.lib, "armBitRevIndexTable1024"))
    assert S.fftLen == 1024 and S.bitRevLength == 1800
    assert C.cast(S.pTwiddle, C.c_void_p).value == tw
    assert C.cast(S.pBitRevTable, C.c_void_p).value == br
    R = dsp.const_instance("arm_rfft_fast_sR_f32_len4096")
    assert R.fftLenRFFT == 4096 and R.Sint.fftLen == 2048


@pytest.mark.parametrize("kind", ["f32", "q31", "q15"])
def test_init_functions_match_reference(dsp, ref, kind):
    """arm_cfft_init_<kind> fills the same fields as the reference's (pointers excepted:
    each library points at its own copy of the tables)."""
    for n in (16, 32, 64, 128, 256, 512, 1024, 2048, 4096, 100):
        S = getattr(dsp, f"arm_cfft_instance_{kind}")()
        st = getattr(dsp, f"arm_cfft_init_{kind}")(S, n)
        Sr = type(S)()
        st_r = ref.fn(f"arm_cfft_init_{kind}")(C.byref(Sr), n)
        assert st == st_r
        if st == 0:
            assert (S.fftLen, S.bitRevLength) == (Sr.fftLen, Sr.bitRevLength)


def test_shipped_library_is_the_default_build(dsp):
    """The in-tree library that tests, smoke() and bench.py load is built with no tuning macro
    (arm_mi355x_version() lists any in brackets, and every bench line prints it as `library`),
    so the measured kernels are the documented defaults."""
    v = dsp.version()
    assert v.startswith("cmsisdsp-mi355x ") and "gfx950" in v
    assert "[" not in v, v
