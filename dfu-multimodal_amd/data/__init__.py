"""Paired RGB + thermal data: the reference's dataset semantics."""
