"""CPU oracle for the placement-scoring path — test infrastructure only (see oracle.py)."""
