#!/bin/bash
set -u
bash scripts/r03/base.sh || exit $?
bash scripts/r03/dkdv.sh || exit $?
bash scripts/r03/km.sh
