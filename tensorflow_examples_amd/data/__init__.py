"""data package."""
