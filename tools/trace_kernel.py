#!/usr/bin/env python3
"""Per-call durations (us) of the kernels whose name contains a pattern, from a rocprofv3
--kernel-trace csv:  python tools/trace_kernel.py <kernel_trace.csv> <pattern> [<pattern> ...]"""
import csv
import sys


def main():
    rows = list(csv.reader(open(sys.argv[1])))
    h = rows[0]
    ki, s, e = h.index("Kernel_Name"), h.index("Start_Timestamp"), h.index("End_Timestamp")
    for pat in sys.argv[2:]:
        w = [(int(x[e]) - int(x[s])) / 1000 for x in rows[1:] if pat in x[ki]]
        print(pat, len(w), "calls, us:", [round(v, 1) for v in w])


if __name__ == "__main__":
    main()
