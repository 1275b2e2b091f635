"""ORACLE — test infrastructure only (never the product path).

CPU restatement of the CSA-Trans attention hot path, used as the parity checker by
``tests/``, by ``__graft_entry__.smoke()`` and as the ``cpu_baseline`` leg of ``bench.py``.
Nothing under ``code-structure-aware-transformer_amd/`` may import this package.

Parity is PINNED: ``tests/golden/*.npz`` were produced by importing the reference itself
(``tools/gen_golden.py``, reference @ /root/reference) and ``tests/test_oracle_golden.py``
checks every function here against them.

Modules
-------
sbm_ref      op-for-op torch-CPU restatement of module/sbm_attn.py + module/STE.py
             (autograd backward, exactly like the reference)
closed_form  fp64 closed-form forward/backward of the same math (the spec the HIP
             kernels implement; cross-checked against sbm_ref autograd)
cse_ref      op-for-op restatement of module/disentangled_attn.py (+ rel/mask build of
             module/csa_trans.py:204-217)
"""
