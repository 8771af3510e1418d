"""Drop-in ``losses`` package (reference losses/)."""
