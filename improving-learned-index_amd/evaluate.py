"""CLI alias mirroring `python -m src.deep_impact.evaluate` (reference evaluate.py:6-18)."""
from .metrics import main

if __name__ == "__main__":
    main()
