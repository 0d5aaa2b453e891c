"""Empty stand-in for the absent ``crimson`` package (only ``sctools.groups`` imports it)."""
picard = None
