"""Drop-in mirrors of the reference tower_code/ modules."""
