"""CPU oracle for the Enhanced-UNet training hot path.

TEST INFRASTRUCTURE ONLY.  Nothing under ``oracle/`` is part of the product:
only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import it, and only as the checker / the timed CPU baseline, never as
the thing measured or shipped.  The product path (``enhanced-unet_amd/eunet``)
never imports this package and fails loudly when its HIP library is missing.

Parity is pinned: ``tests/golden/*.npz`` were produced by importing the
reference (``/root/reference/{models,train_eval}.py``) in the build container
(``tests/golden/gen_golden.py``), and ``tests/test_oracle.py`` checks this
restatement against them.
"""
