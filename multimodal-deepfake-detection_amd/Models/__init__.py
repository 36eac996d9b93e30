"""Reference-compatible model package (``from Models.XceptionLSTMV import XceptionLSTMV``)."""
