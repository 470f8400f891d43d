"""CPU ORACLE — TEST INFRASTRUCTURE ONLY.

A plain-PyTorch-CPU / numpy restatement of the reference's reverse-diffusion
enhancement path (yh-jun/SNR-Aligned_diffSE, `sgmse-bbed/sgmse/...`), used as the
checker for the HIP product path and as the timed `cpu_baseline` leg of bench.py.

Rules (see DESIGN.md "Oracle"):
  * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may import this
    package.  The product package (snr-aligned_diffse_amd/) never imports it and has no
    CPU fallback: its ops raise when the HIP library is missing.
  * Every function cites the reference file:line it restates.
  * Pinning: the restatement is checked against golden vectors produced by running the
    reference's own modules in the build container (tools/gen_golden.py ->
    tests/golden/*.npz); tests/test_oracle_golden.py holds those checks.  The reference
    has no tests of its own, so these goldens are the only pin; glue that
    lives in modules the reference cannot import here (model.py, data_module.py) is
    restated from source text and pinned through the same goldens' restated glue.
"""
