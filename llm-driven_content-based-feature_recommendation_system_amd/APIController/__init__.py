"""Drop-in mirror of the reference APIController/ package."""
