"""Print glibc's __logf_data (the table the host logf uses) from the installed libm.

The constants of cmsis-dsp_amd/csrc/host_logf.hpp come from here: struct logf_data { struct
{double invc, logc;} tab[16]; double ln2; double poly[3]; } is located in libm's read-only
data by its ln2 word followed by poly[0] ~ -0.25.  glibc 2.35 (Ubuntu 2.35-0ubuntu3.x) is the
version pinned by this image; tools/logf_check.cpp then proves the restatement equal to the
host logf for every float input."""
import struct
import sys

LIBM = sys.argv[1] if len(sys.argv) > 1 else "/lib/x86_64-linux-gnu/libm.so.6"
b = open(LIBM, "rb").read()
ln2 = struct.pack("<d", float.fromhex("0x1.62e42fefa39efp-1"))
i = 0
while (i := b.find(ln2, i)) >= 0:
    poly = struct.unpack("<3d", b[i + 8:i + 32])
    if abs(poly[0] + 0.25) < 0.01:
        tab = struct.unpack("<32d", b[i - 256:i])
        for k in range(16):
            print(f"{{{tab[2 * k].hex()}, {tab[2 * k + 1].hex()}}},")
        print("ln2", struct.unpack("<d", ln2)[0].hex(), "poly", [p.hex() for p in poly])
        break
    i += 1
else:
    sys.exit("logf table not found")
