"""``llama-server`` compatible entry point for the GGUF tier: the chart runs
``command: [hipserve-llama-server]`` with the reference's args
``--host 0.0.0.0 --port 8080 --model <path.gguf> --alias <name>``
(ramalama-models/helm-chart/templates/model-deployments.yaml:26-35)."""
from .cli import main as _main


def main(argv=None):
    return _main(argv, prog="llama-server")


if __name__ == "__main__":
    main()
