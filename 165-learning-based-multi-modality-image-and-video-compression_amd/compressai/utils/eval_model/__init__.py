"""``python -m compressai.utils.eval_model`` (reference: compressai/utils/eval_model/)."""
