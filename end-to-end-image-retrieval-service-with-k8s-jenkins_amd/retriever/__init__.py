"""Retrieve helpers (mirror of reference ``retriever/``)."""
