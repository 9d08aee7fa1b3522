"""CPU oracle for the mme hot path — TEST INFRASTRUCTURE ONLY.

Plain numpy / PyTorch-CPU restatements of the reference's algorithm, each
function citing the reference file:line (or the third-party source the
reference calls) it follows. It is pinned against golden fixtures generated
from the reference itself (tests/golden/make_goldens.py -> tests/golden/*.npz).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package, and only as the CHECKER (or the timed CPU baseline) —
never as the thing measured or shipped. The product path (mme) never imports
it and fails loudly without libmme.
"""
