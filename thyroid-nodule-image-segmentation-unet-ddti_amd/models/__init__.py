"""Mirror of the reference's ``models`` package for the HIP path (models/model.py:UNet,
models/loss.py losses).  Only models.model.UNet is on the accelerated hot path."""
