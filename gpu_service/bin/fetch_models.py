"""Check (and optionally fetch) the HF checkpoints gpu_service is configured to serve
(reference gpu_service/bin/fetch_models.py).  Engine presets with random weights need nothing."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from gpu_service.models import embedder_models, provider_models
    from django_assistant_bot_amd.models.configs import decoder_config, encoder_config

    ap = argparse.ArgumentParser()
    ap.add_argument("--download", action="store_true", help="download missing checkpoints (needs network)")
    args = ap.parse_args()
    missing = 0
    for name in embedder_models + provider_models:
        try:
            (encoder_config if name in embedder_models else decoder_config)(name)
            print(f"{name}: engine preset (random-init weights unless a checkpoint path is given)")
            continue
        except KeyError:
            pass
        if os.path.isdir(name):
            print(f"{name}: local checkpoint")
            continue
        try:
            from huggingface_hub import snapshot_download
            path = snapshot_download(name, local_files_only=True)
            print(f"{name}: cached at {path}")
        except Exception:
            if args.download:
                from huggingface_hub import snapshot_download
                print(f"{name}: downloading ...")
                snapshot_download(name)
            else:
                print(f"{name}: MISSING")
                missing += 1
    sys.exit(1 if missing else 0)


if __name__ == "__main__":
    main()
