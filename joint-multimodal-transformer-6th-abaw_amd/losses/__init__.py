"""HIP-backed drop-in replacements for the reference's losses/ package."""
