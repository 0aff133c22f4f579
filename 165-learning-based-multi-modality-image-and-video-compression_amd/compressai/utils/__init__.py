"""Evaluation utilities (reference: compressai/utils/)."""
