"""Mirror of the reference's ``models`` package for the HIP path (models/model.py:UNet,
models/mod.py:UNet, models/loss.py losses)."""
