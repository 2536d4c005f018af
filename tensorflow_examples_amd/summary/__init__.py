"""summary package."""
