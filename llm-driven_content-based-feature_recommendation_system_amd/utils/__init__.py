"""Drop-in mirror of the reference utils/ package (contracts only)."""
