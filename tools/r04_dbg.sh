cd $GRAFT_REPO_ROOT
LGBM_AMD_KTRACE=1 timeout -k 10 120 python -u tools/debug/self_check.py 2>&1 | grep -v "^round\|^plan" | cut -c1-400 | head -40
