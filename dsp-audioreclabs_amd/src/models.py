"""Drop-in for the reference's src/models.py on MI355X (KNN on the device)."""
