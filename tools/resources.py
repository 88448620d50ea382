"""VGPRs / scratch / occupancy per kernel from hipcc -Rpass-analysis=kernel-resource-usage on stdin."""
import re
import sys

cur, vals = None, {}
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur, vals = m.group(1), {}
        continue
    m = re.search(r"remark:\s+(VGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]): (\d+)", line)
    if m and cur:
        key = m.group(1).split()[0]
        vals[key] = m.group(2)
        if key == "Occupancy":
            print("%-72s vgpr=%s scratch=%s occ=%s" % (cur[:72], vals.get("VGPRs"), vals.get("ScratchSize"), vals[key]))
