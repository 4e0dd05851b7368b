"""Drop-in `models` package of the DFU fusion path on MI355X (the reference's surface:
models/encoders.py, models/fusion.py, models/models.py, models/classifier.py)."""
