"""CPU oracle -- TEST INFRASTRUCTURE ONLY.

A NumPy restatement of the reference's TDA response hot path
(Quantum-Chemistry-Group-BNU/XTDDFT), used exclusively as the checker:
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import it.  The product path (``xtddft_amd``) never imports, calls or
falls back to anything here.

Parity status (see DESIGN.md section "Oracle"):
  The reference cannot be imported or run in this environment (PySCF and
  opt_einsum are absent; XSF_TDA.py:1137 does not parse).  The only known
  answers it ships are notebook outputs for real molecules, which need an
  integral / grid / SCF stack this round does not have.  The operator-level
  oracle is therefore **parity unpinned** against reference outputs; it is
  pinned internally by two independent restatements of two different
  reference code paths (the Davidson ``vind`` AO route vs the explicit-A
  ``full_diag`` / ``get_Amat`` MO-integral route) agreeing to round-off.

Modules:
  engines    -- AO-route J/K (DF) and XC response (PySCF nr_uks_fxc /
                nr_uks_fxc_sf_tda semantics).
  xtda       -- XTDA._gen_tda_operation / vind / hdiag / init guess / precond
                (XTDA.py:482-744) and the explicit A of full_diag (XTDA.py:56-400).
  sf_tda     -- SF_TDA.gen_tda_operation_sf (SF_TDA.py:162-286) + explicit A
                (SF_TDA.py:448-560, 624-804).
  xsf_tda    -- XSF_TDA.gen_tda_operation_sf + preconditioner + OO compression
                (XSF_TDA.py:397-427, 859-1290) + explicit A (XSF_TDA.py:265-395).
  davidson   -- davidson1 (Davidson.py:21-298 with PySCF linalg_helper semantics).
  utils      -- order_pyscf2my / so2st / st2so (utils.py:44-122).
"""
