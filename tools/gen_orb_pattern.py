"""Regenerate include/odo_orb_pattern.h from the reference's ORB pattern table.

Run in the build container only (reads /root/reference, which is absent on
the GPU box). The table is constant data (OpenCV's learned ORB pattern).
"""
import re
import sys

src = open(sys.argv[1] if len(sys.argv) > 1 else
           '/root/reference/Features/orbextractor.cpp').read()
m = re.search(r'bit_pattern_31_\[256 \* 4\] = \{(.*?)\};', src, re.S)
body = re.sub(r'/\*.*?\*/', '', m.group(1))
vals = [int(v) for v in re.findall(r'-?\d+', body)]
assert len(vals) == 1024
print(','.join(map(str, vals)))
