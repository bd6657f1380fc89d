"""Drop-in mirror of the reference temp_model/ (rerank) package."""
