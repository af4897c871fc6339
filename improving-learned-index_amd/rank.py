"""CLI alias mirroring `python -m src.deep_impact.rank` (reference rank.py:6-22)."""
from .ranker import main

if __name__ == "__main__":
    main()
