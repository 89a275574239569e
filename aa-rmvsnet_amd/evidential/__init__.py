"""Drop-in ``evidential`` package (reference: evidential/models.py)."""
