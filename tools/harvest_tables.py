#!/usr/bin/env python3
"""Harvest the reference's CommonTables data into binary blobs for the product library.

The twiddle and bit-reversal tables of CMSIS-DSP cannot be regenerated from formulas
bit-for-bit (f32 differs from float(cos) in 43/2048 entries at N=1024,
q31 matches no rounding rule), so the exact words are read out of the reference build
(`oracle/_ref/libcmsisdsp_ref.so`, compiled from
/root/reference/Source/CommonTables/arm_common_tables.c by `oracle/ref.mk`) and written
as raw little-endian blobs under cmsis-dsp_amd/tables/, with a sha256 manifest.
The product embeds the blobs with `.incbin` (cmsis-dsp_amd/csrc/tables_data.S), so the
data symbols keep the reference's names (`twiddleCoef_1024`, ...) for drop-in apps.

Run in this container only (needs the reference build):  python tools/harvest_tables.py
"""
import ctypes
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libcmsisdsp_ref.so")
OUT = os.path.join(ROOT, "cmsis-dsp_amd", "tables")

SIZES = [16, 32, 64, 128, 256, 512, 1024, 2048, 4096]
RFFT_SIZES = [32, 64, 128, 256, 512, 1024, 2048, 4096]

# bit-reversal table lengths: Include/arm_common_tables.h:181-235
BITREV_LEN = {16: 20, 32: 48, 64: 56, 128: 208, 256: 440, 512: 448,
              1024: 1800, 2048: 3808, 4096: 4032}
BITREV_FIXED_LEN = {16: 12, 32: 24, 64: 56, 128: 112, 256: 240, 512: 480,
                    1024: 992, 2048: 1984, 4096: 4032}


def tables():
    """(symbol, ctype, count) for every table on the hot path (arm_common_tables.h:61-236)."""
    t = []
    for n in SIZES:
        t.append((f"twiddleCoef_{n}", ctypes.c_float, 2 * n))
        t.append((f"twiddleCoef_{n}_q31", ctypes.c_int32, 3 * n // 2))
        t.append((f"twiddleCoef_{n}_q15", ctypes.c_int16, 3 * n // 2))
        t.append((f"armBitRevIndexTable{n}", ctypes.c_uint16, BITREV_LEN[n]))
        t.append((f"armBitRevIndexTable_fixed_{n}", ctypes.c_uint16, BITREV_FIXED_LEN[n]))
    for n in RFFT_SIZES:
        t.append((f"twiddleCoef_rfft_{n}", ctypes.c_float, n))
    return t


class CfftInst(ctypes.Structure):
    _fields_ = [("fftLen", ctypes.c_uint16), ("pTwiddle", ctypes.c_void_p),
                ("pBitRevTable", ctypes.c_void_p), ("bitRevLength", ctypes.c_uint16)]


def main():
    if not os.path.exists(REF_SO):
        sys.exit(f"{REF_SO} missing: run `make -f oracle/ref.mk` first")
    lib = ctypes.CDLL(REF_SO)
    os.makedirs(OUT, exist_ok=True)
    manifest = {"source": "reference CommonTables via oracle/_ref/libcmsisdsp_ref.so",
                "tables": {}, "bitRevLength": {}}
    for name, ct, count in tables():
        arr = (ct * count).in_dll(lib, name)
        raw = bytes(arr)
        with open(os.path.join(OUT, name + ".bin"), "wb") as f:
            f.write(raw)
        manifest["tables"][name] = {"ctype": ct.__name__, "count": count,
                                    "bytes": len(raw),
                                    "sha256": hashlib.sha256(raw).hexdigest()}
    # cross-check the table lengths against the reference's own const structs
    for kind in ("f32", "q31", "q15"):
        for n in SIZES:
            s = CfftInst.in_dll(lib, f"arm_cfft_sR_{kind}_len{n}")
            want = BITREV_LEN[n] if kind == "f32" else BITREV_FIXED_LEN[n]
            assert s.fftLen == n and s.bitRevLength == want, (kind, n, s.bitRevLength)
            manifest["bitRevLength"][f"{kind}_{n}"] = s.bitRevLength
    with open(os.path.join(OUT, "MANIFEST.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print(f"wrote {len(manifest['tables'])} tables to {OUT}")


if __name__ == "__main__":
    main()
