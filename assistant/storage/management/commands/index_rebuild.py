"""``manage.py index_rebuild`` -- reload the HBM vector indexes from the database."""
from django.core.management import BaseCommand

from assistant.storage.index import get_index_service
from assistant.storage.models import Document, Question, Sentence


class Command(BaseCommand):
    help = "Rebuild the in-HBM vector indexes from the database"

    def handle(self, *args, **options):
        svc = get_index_service()
        for model, field in ((Question, "embedding"), (Sentence, "embedding"), (Document, "content_embedding")):
            n = svc.rebuild(model, field)
            self.stdout.write(f"{model._meta.label}.{field}: {n} rows ({svc.backend_name})")
