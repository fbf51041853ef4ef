"""CPU oracle for the DDTI UNet hot path.

TEST INFRASTRUCTURE ONLY.  Nothing under ``oracle/`` is part of the product:
only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` may import it, and only as the checker (never as the thing that is
measured or shipped).  The product path (``unet_hip``) never imports this
package and fails loudly when its HIP library is missing.

Contents
--------
* ``weights``      - counter-hash (splitmix64) parameter / input generator, so
                     every fixture can be regenerated on the GPU box with no
                     reference code.
* ``unet_ref_cpu`` - torch-CPU restatement of ``models/model.py:UNet``, the
                     losses of ``models/loss.py`` + ``nn.BCEWithLogitsLoss``,
                     the training step of ``utils/trainer.py:81-93`` and the
                     single-tensor AdamW update torch runs on CPU.

Parity pin: ``tools/gen_golden.py`` imports the real reference (in the build
container only) and writes ``tests/golden/*.npz``; ``tests/test_oracle.py``
checks this restatement against those fixtures.
"""
