"""CPU oracle (test infrastructure only; see oracle/unet_ref.py header)."""
