"""Stand-in ``isaacgym`` package used ONLY to import the reference task module
in the build container while generating golden fixtures (tests/golden/make_golden.py).
Never imported by the product path."""
