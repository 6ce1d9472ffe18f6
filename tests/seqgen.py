"""Test-side re-export of the seeded generators (taxi2_amd/synth.py)."""

from taxi2_amd.synth import family_sequences, mutate, random_sequences  # noqa: F401
