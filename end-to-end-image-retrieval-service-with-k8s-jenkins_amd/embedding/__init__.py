"""Embedding service (mirror of reference ``embedding/``)."""
