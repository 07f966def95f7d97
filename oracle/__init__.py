"""CPU oracle for the gnnea hot path — TEST INFRASTRUCTURE ONLY.

Restatements of the reference algorithms (HestiaSky/GNN-MTL) in fp64 numpy / torch-CPU, each
function citing the reference file:line it follows.  Pinned against the golden fixtures that
tests/golden/gen_golden.py produced by running the reference itself (tests/test_oracle.py).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package,
and only as the checker / the timed CPU baseline — never as a product path.
"""
