"""Test-infrastructure oracle (CPU, fp32).  Never imported by the product path."""
