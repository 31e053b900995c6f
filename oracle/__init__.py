"""TEST INFRASTRUCTURE ONLY — the CPU parity oracle. Importable by tests/, smoke() and the
bench.py cpu_baseline leg; never by the product (ghex_amd)."""
