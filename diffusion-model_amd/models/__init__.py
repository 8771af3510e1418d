"""Drop-in replacements of the reference's ``models`` package (hot-path networks)."""
