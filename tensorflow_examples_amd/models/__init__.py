"""models package."""
