# Round profile at HEAD: GPU tests + smoke + kernel traces + PMC traffic + bench line
# (tools/gpu_round.sh), then the headline SQ counter passes (tools/pmc_headline.sh).
# Usage: bash tools/gpu_profile_session.sh <tag>
set -o pipefail
TAG=${1:-r05p}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/gpu_round.sh "$TAG" || exit 1
bash tools/pmc_headline.sh "${TAG}_hl" || exit 1
cp "gpurun_out/pmc_${TAG}_hl/summary.json" "gpurun_out/${TAG}_hl_pmc.json"
ls profiles | grep "$TAG"
