"""ckpt package."""
