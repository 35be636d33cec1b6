"""``manage.py search <query>`` -- broad document search over questions or sentences.  Fixes the
reference command's stale call (it passed no QuerySet and an unknown ``field`` argument)."""
import asyncio

from django.core.management import BaseCommand

from assistant.rag.services.search_service import embedding_search
from assistant.storage.models import Question, Sentence


class Command(BaseCommand):
    help = "Search documents by embedding similarity"

    def add_arguments(self, parser):
        parser.add_argument("query", type=str)
        parser.add_argument("--field", type=str, choices=("sentences", "questions"), default="questions")
        parser.add_argument("--bot", type=str, default=None, help="restrict to a bot codename")
        parser.add_argument("--max-scores-n", default=5, type=int)
        parser.add_argument("--n", default=10, type=int)

    def handle(self, *args, **options):
        model = Question if options["field"] == "questions" else Sentence
        qs = model.objects.all()
        if options["bot"]:
            qs = qs.filter(document__wiki__bot__codename=options["bot"])
        results = asyncio.run(embedding_search(options["query"], qs, max_scores_n=options["max_scores_n"],
                                               top_n=options["n"]))
        for document, score in results:
            self.stdout.write(f"{document.id}  {score:.4f}  {document.name}")
