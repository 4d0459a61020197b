"""CPU oracle for the FD perturbation-evaluation hot path -- TEST INFRASTRUCTURE ONLY.

This package is a plain numpy / torch-CPU restatement of the reference algorithm
(nexus-rl/dfd-starter, mounted read-only at /root/reference in the build container).
Every function cites the reference file:line it follows.

Rules (DESIGN.md "Oracle"):
  * Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
    leg may import anything from here, and only as the CHECKER / the timed CPU
    baseline -- never as the product path.  The product (``dfd-starter_amd``) never
    imports ``oracle`` and fails loudly when its HIP library is missing.
  * Parity is pinned: ``tests/golden/make_golden.py`` imports the reference itself
    in the build container and writes the fixtures under ``tests/golden/``;
    ``tests/test_oracle_golden.py`` checks this restatement against them.
  * Third-party arithmetic the reference relies on (numpy legacy ``RandomState``
    MT19937 / polar Box-Muller, OpenBLAS sdot/dgemv, torch CPU nn ops) is used
    here directly, exactly as the reference uses it.
"""
