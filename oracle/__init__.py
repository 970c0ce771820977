"""CPU oracle for the Swin-unrolled cine reconstruction hot path.

TEST INFRASTRUCTURE ONLY.  Nothing under ``oracle/`` is part of the product:
only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import it, and only as the checker / the timed CPU baseline.  The
product path (``dl-swin-gan_amd/dl_cs``) never imports this package.

* ``dlcs_oracle`` -- plain PyTorch-CPU fp32 / complex64 functional restatement
  of the reference path (SenseModel, Swin regularizer, unrolled PGD, metrics).
* ``windex``      -- numpy restatement of the integer bookkeeping
  (window partition / reverse permutations, cyclic shift, shift mask labels,
  relative-position index, ``get_window_size``).
* ``recipe``      -- deterministic weight / input recipes shared by the golden
  generator (run in the survey container against the reference) and the tests
  (run anywhere), so no multi-MB weight files are stored.

Parity pin: every function here is checked against golden vectors produced by
importing the reference itself (``tests/golden/make_golden.py``).
"""
