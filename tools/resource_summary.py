#!/usr/bin/env python3
"""Summarise `make resource-usage` remarks (one line per kernel: VGPRs, scratch, occupancy, LDS,
spills) so two builds' register allocations can be diffed.  Usage: resource_summary.py REMARKS.txt"""
import re
import sys

rows, cur = {}, None
for line in open(sys.argv[1]):
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[[^\]]*\])?: (\S+) \[", line)
    if m and cur:
        rows[cur][m.group(1)] = m.group(2)
for k in sorted(rows):
    r = rows[k]
    print(f"{k[:90]:90s} v{r.get('VGPRs', '?'):>4} s{r.get('ScratchSize', '?'):>5} occ{r.get('Occupancy', '?'):>2} "
          f"lds{r.get('LDS Size', '?'):>6} vsp{r.get('VGPRs Spill', '?'):>4}")
