"""Computer-vision example components (reference ``examples/vision``)."""
