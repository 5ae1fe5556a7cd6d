"""CPU parity checker — TEST INFRASTRUCTURE ONLY (tests/, smoke(), bench cpu_baseline)."""
