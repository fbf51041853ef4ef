"""Mirror of the reference's ``utils`` package: Trainer (utils/trainer.py), bookkeeping
(utils/utils.py) and the paired transforms main.py needs (utils/transforms.py)."""
