"""HIP-backed drop-in replacements for the reference's models/ package (fusion models only;
the frozen backbones of models/tsav.py etc. are out of scope)."""
