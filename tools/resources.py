"""Summarize hipcc -Rpass-analysis=kernel-resource-usage output per kernel."""
import re
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "cppserver_amd/_build/asm/resource-usage.txt"
rows, cur = [], None
KEYS = [("TotalSGPRs", "sgpr"), ("VGPRs", "vgpr"), ("ScratchSize", "scratch"), ("Occupancy", "occ"), ("LDS Size", "lds")]
for line in open(path):
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": re.sub(r"^_ZN3wsg\d+", "", m.group(1))[:28]}
        rows.append(cur)
        continue
    if cur is None or "remark" not in line:
        continue
    for key, label in KEYS:
        m = re.search(r"(?:^|\s)" + re.escape(key) + r"(?: \[[^\]]*\])?:\s*(\d+)", line)
        if m and label not in cur:
            cur[label] = int(m.group(1))
for r in rows:
    print("%-30s sgpr=%-4s vgpr=%-4s scratch=%-4s occ=%-2s lds=%s" % (
        r["name"], r.get("sgpr"), r.get("vgpr"), r.get("scratch"), r.get("occ"), r.get("lds")))
