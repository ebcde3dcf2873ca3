"""Scenarios: MComCustom (reference scenarios/custom.py) and the batched scenario registry."""
