#!/usr/bin/env bash
# One-command provisioner for an MI355X Kubernetes node + the llm-d-compatible serving
# stack (CLI-compatible with the reference: deploy | cleanup | help; no argument = deploy).
#
#   AKAP_NODE_HOST=10.0.0.5 ./deploy-k8s-cluster.sh deploy     # bare-metal 8x MI355X
#   AKAP_DEPLOY_MODE=kind    ./deploy-k8s-cluster.sh deploy     # CPU-only rehearsal on kind
#   ./deploy-k8s-cluster.sh cleanup                             # tear down what deploy created
#
# Environment: AKAP_CONFIG (default config/cluster.yaml), AKAP_NODE_HOST, AKAP_DEPLOY_MODE,
# AKAP_VALUES_PRESET (slim|pd|tp8|moe|kind), AKAP_EXTRA_VARS ("k=v k2=v2"), AKAP_YES=1
# (no confirmation prompt on cleanup), ANSIBLE_PLAYBOOK (binary override).
set -euo pipefail

HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
CONFIG="${AKAP_CONFIG:-$HERE/config/cluster.yaml}"
PLAYBOOK_BIN="${ANSIBLE_PLAYBOOK:-ansible-playbook}"
PB="$HERE/provision"

usage() {
    cat <<USAGE
Usage: $0 [deploy|cleanup|help]

Commands:
  deploy    Provision the MI355X node (ROCm, CRI-O, kubeadm, AMD device plugin, storage,
            Prometheus), deploy the serving stack (gateway + engine pods), smoke-test the
            OpenAI API through the gateway, and wire the OpenTelemetry metrics pipeline.
  cleanup   Reset the node(s) recorded in gpu-inventory-*.ini and remove local state.
  help      Show this message.
USAGE
    exit "${1:-1}"
}

extra_args() {
    local args=(-e "@$CONFIG")
    [[ -n "${AKAP_NODE_HOST:-}" ]] && args+=(-e "node_host=$AKAP_NODE_HOST")
    [[ -n "${AKAP_DEPLOY_MODE:-}" ]] && args+=(-e "deploy_mode=$AKAP_DEPLOY_MODE")
    [[ -n "${AKAP_VALUES_PRESET:-}" ]] && args+=(-e "values_preset=$AKAP_VALUES_PRESET")
    if [[ -n "${AKAP_EXTRA_VARS:-}" ]]; then
        for kv in $AKAP_EXTRA_VARS; do args+=(-e "$kv"); done
    fi
    printf '%s\n' "${args[@]}"
}

run_pb() {  # run_pb <playbook> [inventory]
    local pb="$1" inv="${2:-}"
    local -a xs
    mapfile -t xs < <(extra_args)
    echo ">>> ${pb##*/}"
    if [[ -n "$inv" ]]; then
        "$PLAYBOOK_BIN" -i "$inv" "${xs[@]}" "$pb"
    else
        "$PLAYBOOK_BIN" "${xs[@]}" "$pb"
    fi
}

newest() {  # newest file matching a glob, by mtime; empty if none
    local f
    f="$(ls -t $1 2>/dev/null | head -n 1 || true)"
    printf '%s' "$f"
}

deploy_cluster() {
    echo "=== Deploying the MI355X Kubernetes node + serving stack ==="
    run_pb "$PB/inventory-baremetal.yaml"
    local inv
    inv="$(newest 'gpu-inventory-*.ini')"
    if [[ -z "$inv" ]]; then
        echo "Error: no gpu-inventory-*.ini was produced" >&2
        exit 1
    fi
    echo "Using inventory file: $inv"
    run_pb "$PB/rocm-node.yaml" "$inv"
    run_pb "$PB/kubernetes-single-node.yaml" "$inv"
    run_pb "$PB/llm-d-deploy.yaml" "$inv"
    run_pb "$PB/llm-d-test.yaml" "$inv"
    run_pb "$PB/otel-observability-setup.yaml" "$inv"

    echo ""
    echo "=== Node Information ==="
    local details
    details="$(newest 'instance-*-details.txt')"
    if [[ -n "$details" ]]; then
        for key in "Instance ID" "Instance Name" "Instance Type" "Public IP" "Private IP" "GPUs"; do
            grep -m1 "^$key:" "$details" || true
        done
        echo ""
        echo "SSH Access:"
        grep -m1 "ssh -i" "$details" || true
        echo ""
        echo "Full details saved to: $details"
    else
        echo "Warning: no instance-*-details.txt found"
    fi
}

cleanup_instances() {
    echo "=== Cleaning up MI355X node(s) ==="
    if ! ls gpu-inventory-*.ini >/dev/null 2>&1; then
        echo "No inventory files found. Nothing to cleanup."
        exit 0
    fi
    if [[ "${AKAP_YES:-0}" != "1" && -t 0 ]]; then
        echo "Inventories: $(ls gpu-inventory-*.ini | tr '\n' ' ')"
        read -r -p "Reset these node(s) and delete local state? [y/N] " ans
        [[ "$ans" == "y" || "$ans" == "Y" ]] || { echo "Aborted."; exit 1; }
    fi
    run_pb "$PB/cleanup-instance.yaml"
    echo "Cleanup complete!"
}

case "${1:-}" in
    deploy)
        shift
        if [[ $# -ne 0 ]]; then
            echo "Deploy command doesn't accept additional arguments" >&2
            usage 1
        fi
        deploy_cluster
        ;;
    cleanup)
        shift
        cleanup_instances
        ;;
    -h|--help|help)
        usage 0
        ;;
    "")
        deploy_cluster
        ;;
    *)
        echo "Unknown command: $1" >&2
        usage 1
        ;;
esac
