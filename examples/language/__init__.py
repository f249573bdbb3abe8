"""Language-model example components (reference ``examples/language``)."""
