"""python -m benchmark_dolfinx_amd == bench_dolfinx."""
from .cli import main

raise SystemExit(main())
