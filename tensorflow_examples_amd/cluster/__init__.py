"""cluster package."""
