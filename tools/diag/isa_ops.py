#!/usr/bin/env python3
"""Memory-instruction census of kernels in a device assembly file (hipcc --cuda-device-only -S):
  python tools/diag/isa_ops.py file.s [name-substring]"""
import collections
import re
import sys


def main(path, pat=""):
    s = open(path).read()
    for m in re.finditer(r'\n(_Z\w+):\s*;[^\n]*\n(.*?)\n\s*s_endpgm', s, re.S):
        name, body = m.group(1), m.group(2)
        if pat not in name:
            continue
        c = collections.Counter(re.findall(r'^\s+(flat_\w+|global_\w+|ds_\w+|buffer_\w+|s_waitcnt)', body, re.M))
        vg = re.search(r'\.vgpr_count:\s+(\d+)', s[m.end():m.end() + 20000])
        print(name[:90])
        print("  ", sorted(c.items(), key=lambda x: -x[1])[:24])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
