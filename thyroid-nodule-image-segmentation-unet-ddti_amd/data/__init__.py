"""Mirror of the reference's ``data`` package (data/data_loader.py)."""
