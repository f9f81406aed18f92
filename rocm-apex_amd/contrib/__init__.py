"""Contrib modules (reference apex/contrib)."""
