"""Ingest helpers (mirror of reference ``ingesting/``)."""
