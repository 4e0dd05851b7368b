"""Test-only CPU oracle (see oracle/torch_ref.py). Never imported by the product package."""
