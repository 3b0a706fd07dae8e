set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=r03m_n17 CFG="--n 131072" bash tools/phase_cost.sh || exit 1
TAG=r03m_c2 CFG="--config c2" bash tools/phase_cost.sh || exit 1
TAG=r03m_c3 CFG="--config c3" INF=8 bash tools/phase_cost.sh || exit 1
