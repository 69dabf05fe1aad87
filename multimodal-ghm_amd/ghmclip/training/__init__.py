"""Training entry points: python -m ghmclip.training.train_CLIP (reference CLI)."""
