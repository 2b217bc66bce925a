# r05: GPU suite, per-kernel SQ instruction mix, pass-scheduling A/B (one call)
bash tools/r05_tests_pmc.sh && bash tools/r05_ab3.sh
