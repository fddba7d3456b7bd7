"""MI355X (gfx950) drop-in for the reference's src/ package (Hypersonic-cpu/DSP-AudioRecLabs).

Module surface kept from the reference: audio_processing, feature_extraction, models.
Batched device API: src.pipeline.  C ABI: include/dsp_audiorec.h.
"""
__version__ = "1.0.0"
