"""Test-infrastructure oracle (CPU restatement of the reference update path).
Never imported by the product package `mjrl_amd`; see oracle/npg_cpu.py."""
