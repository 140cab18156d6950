#!/usr/bin/env python3
"""Regenerate antpolarcodes_amd/csrc/host/nr_reliability.inc (build container only).

Reads the 3GPP TS 38.212 polar reliability sequence from the reference's
header /root/reference/include/polarcode/construction/fiveGList.h and writes its
inverse permutation (rank of each sub-channel index).  Not used at run time.
"""
import re
import sys

REF = "/root/reference/include/polarcode/construction/fiveGList.h"
OUT = "antpolarcodes_amd/csrc/host/nr_reliability.inc"


def main():
    src = open(REF).read()
    body = src[src.index("RELIABILITY_TABLE = {") + len("RELIABILITY_TABLE = {"):]
    seq = [int(x) for x in re.findall(r"\d+", body[:body.index("}")])]
    if len(seq) != 1024 or sorted(seq) != list(range(1024)):
        sys.exit("unexpected table shape")
    rank = [0] * 1024
    for r, i in enumerate(seq):
        rank[i] = r
    lines = [l for l in open(OUT).read().split("\n") if l.startswith("//")]
    for k in range(0, 1024, 16):
        lines.append("    " + ", ".join("%4d" % v for v in rank[k:k + 16]) + ",")
    open(OUT, "w").write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
