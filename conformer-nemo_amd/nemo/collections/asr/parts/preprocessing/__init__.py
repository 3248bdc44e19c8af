"""Preprocessing (reference nemo/collections/asr/parts/preprocessing)."""
