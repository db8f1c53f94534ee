"""Resource report of the kernels in a device .s file (hipcc --cuda-device-only -S):
VGPRs, AGPR offset, scratch bytes, vmcnt waits (and how many drain to 0), MFMA count.
Usage: python tools/kasm.py file.s [name-substring]"""
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else ""
for m in re.finditer(r"^(_Z\S+):[^\n]*\n(.*?)^\.Lfunc_end", s, re.M | re.S):
    name, body = m.group(1), m.group(2)
    if pat not in name:
        continue
    md = re.search(r'\.amdhsa_kernel ' + re.escape(name) + r'\n(.*?)\.end_amdhsa_kernel', s, re.S)
    if not md:
        continue
    md = md.group(1)
    g = lambda k: re.search(r'\.amdhsa_' + k + r' (\d+)', md).group(1)
    n0 = len(re.findall(r'vmcnt\(0\)', body))
    nv = len(re.findall(r's_waitcnt vmcnt', body))
    nm = len(re.findall(r'v_mfma', body))
    print(f"{name[:70]:70s} vgpr {g('next_free_vgpr'):>3} acc {g('accum_offset'):>3} "
          f"scratch {g('private_segment_fixed_size'):>4} vmcnt0 {n0:>3} vmcnt {nv:>3} mfma {nm:>4}")
