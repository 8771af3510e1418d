"""CPU oracle for the CFG denoising loop — TEST INFRASTRUCTURE ONLY.

This package is a CPU restatement (plain PyTorch-CPU functional ops, fp32,
NCHW) of the reference's hot path.  Every function cites the reference
file:line it follows.  It exists to *check* the MI355X path:

  * only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
    ``cpu_baseline`` leg may import it;
  * the product (``diffusion-model_amd/``) never imports it, and fails
    loudly if its HIP library is missing instead of falling back here.

Parity pinning: the oracle is checked against golden vectors produced by
importing the reference itself in the build container
(``tests/golden/make_golden.py`` -> ``tests/golden/*.npz``); see
``tests/test_oracle_golden.py``.
"""
