"""CPU ORACLE — test infrastructure, not product.

numpy restatements of the reference forward passes (InformerStack / Informer,
InformerLSQ, Transformer) and the NMSE reductions, each function citing the
reference file:line it follows.  Pinned against fixtures produced by running the
reference itself (tests/golden/make_golden.py).  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package;
the engine (channelestimationtransformer_amd) never does.
"""
