"""Structured grids (ghex.structured)."""
