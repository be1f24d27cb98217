// mini_xml.h -- TEST INFRASTRUCTURE (oracle side).  A ~100-line XML element reader used by the
// CPU oracle and by the reference harness to read XMLBIF files.  It replaces the role tinyxml2
// plays for the reference (`include/XMLBIFParser.h:8`, `src/XMLBIFParser.cpp:3-24`): only
// elements, their concatenated text and their children in document order are kept; attributes,
// the <?xml ...?> prologue and comments are skipped.  Not used by the product library.
#ifndef FBN_ORACLE_MINI_XML_H
#define FBN_ORACLE_MINI_XML_H

#include <cstdio>
#include <fstream>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

namespace mini_xml {

struct Element {
    std::string name;
    std::string text;  // concatenated character data directly inside this element
    std::vector<std::unique_ptr<Element>> children;

    const Element *first(const std::string &n) const {
        for (auto &c : children)
            if (c->name == n) return c.get();
        return nullptr;
    }
    std::vector<const Element *> all(const std::string &n) const {
        std::vector<const Element *> out;
        for (auto &c : children)
            if (c->name == n) out.push_back(c.get());
        return out;
    }
};

inline std::unique_ptr<Element> parse_string(const std::string &s) {
    auto root = std::make_unique<Element>();
    root->name = "#document";
    std::vector<Element *> stack{root.get()};
    size_t i = 0, n = s.size();
    while (i < n) {
        if (s[i] == '<') {
            if (s.compare(i, 4, "<!--") == 0) {
                size_t e = s.find("-->", i + 4);
                if (e == std::string::npos) throw std::runtime_error("unterminated comment");
                i = e + 3;
                continue;
            }
            if (i + 1 < n && (s[i + 1] == '?' || s[i + 1] == '!')) {
                size_t e = s.find('>', i);
                if (e == std::string::npos) throw std::runtime_error("unterminated declaration");
                i = e + 1;
                continue;
            }
            size_t e = s.find('>', i);
            if (e == std::string::npos) throw std::runtime_error("unterminated tag");
            std::string tag = s.substr(i + 1, e - i - 1);
            i = e + 1;
            if (!tag.empty() && tag[0] == '/') {
                if (stack.size() <= 1) throw std::runtime_error("unbalanced close tag");
                stack.pop_back();
                continue;
            }
            bool self_close = !tag.empty() && tag.back() == '/';
            if (self_close) tag.pop_back();
            size_t sp = tag.find_first_of(" \t\r\n");
            auto el = std::make_unique<Element>();
            el->name = tag.substr(0, sp);
            Element *raw = el.get();
            stack.back()->children.push_back(std::move(el));
            if (!self_close) stack.push_back(raw);
        } else {
            size_t e = s.find('<', i);
            if (e == std::string::npos) e = n;
            stack.back()->text.append(s, i, e - i);
            i = e;
        }
    }
    return root;
}

inline std::unique_ptr<Element> parse_file(const std::string &path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("cannot open " + path);
    std::stringstream ss;
    ss << f.rdbuf();
    return parse_string(ss.str());
}

}  // namespace mini_xml

#endif
