"""manage.py load_csv <file> --bot <codename>  (reference loading/management/commands/load_csv.py)."""
from django.core.management import BaseCommand

from assistant.bot.models import Bot
from assistant.loading.csv_loader import CSVLoader


class Command(BaseCommand):
    help = "Load wiki documents from a CSV file (toc_title, doc_name, doc_content)"

    def add_arguments(self, parser):
        parser.add_argument("file")
        parser.add_argument("--bot", required=True, help="bot codename")

    def handle(self, *args, **options):
        bot = Bot.objects.get(codename=options["bot"])
        n = CSVLoader(bot, filepath=options["file"]).load_sync()
        self.stdout.write(self.style.SUCCESS(f"Loaded {n} wiki documents"))
