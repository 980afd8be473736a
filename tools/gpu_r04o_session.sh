#!/bin/bash
# round-4 session o: the whole -m gpu suite
set -u
cd "$GRAFT_REPO_ROOT"
TAG=r04o STEPS=tests TESTS_LIMIT=1100 PYTEST_FILES="tests" tools/gpu_r04.sh
