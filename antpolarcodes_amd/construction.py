"""Frozen-set construction (host side): Construction::frozen_bits
(src/polarcode/construction/constructor.cpp:41-63 of the reference).

One implementation, in the host C++ library (csrc/host/polarcode_host.cpp), reached
through the pypolar module: "BB" Bhattacharyya bounds (bhattacharrya.cpp:39-82, the
default), "5G" the 3GPP TS 38.212 reliability sequence (fiveGList.cpp:28-37, incl.
SURVEY Q6 for N < 1024), "BE" beta expansion (betaexpansion.cpp:39-78).
"""


def frozen_bits(blockLength, infoLength, designSNR=0.0, constructorType="BB"):
    from .pypolar import frozen_bits as _fb
    return list(_fb(int(blockLength), int(infoLength), float(designSNR), str(constructorType)))
