"""Drop-in replacement for the reference's ``models`` package (see binarized_modules.py)."""
