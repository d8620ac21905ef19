"""Test/bench-only CPU oracle (see stereo_oracle.py header). Never imported by the product package."""
