"""Hugging Face integrations (reference: python/ray/train/huggingface)."""
