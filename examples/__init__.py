"""Example training applications (reference ``examples/``)."""
