"""Drop-in mirror of the reference utils/data_preprocessing package (the reranker input path)."""
