"""Drop-in for the reference's src/feature_extraction.py on MI355X (see audio_processing)."""
